#!/usr/bin/env python3
"""Kernel-trace timeline summary (rocprofv3 --kernel-trace --output-format csv): over the window
from the first to the last detection kernel, the time fractions with 0, 1, 2, ... detection
kernels in flight, and per kernel name the count and the median / p90 / max duration.

usage: kernel_overlap.py <kernel_trace.csv>"""
import csv
import sys
from collections import defaultdict

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
det, other = [], defaultdict(list)
queues = defaultdict(lambda: defaultdict(int))
for r in rows:
    queues[r['Queue_Id']][r['Kernel_Name'][:24]] += 1
    a, b = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    name = r['Kernel_Name'].replace('(anonymous namespace)::', '')
    if name.startswith('ccd_detect'):
        det.append((a, b))
    else:
        other[name[:60]].append((b - a) * 1e-6)
det.sort()
lo, hi = det[0][0], max(b for _, b in det)
ev = sorted([(a, 1) for a, _ in det] + [(b, -1) for _, b in det])
frac, cur, last = defaultdict(float), 0, lo
for t, d in ev:
    frac[cur] += t - last
    cur += d
    last = t
span = hi - lo
print('detections %d, window %.1f ms, durations median %.2f ms' % (
    len(det), span * 1e-6, float(np.median([(b - a) * 1e-6 for a, b in det]))))
print('in flight: ' + ', '.join('%d: %.3f' % (k, v / span) for k, v in sorted(frac.items())))
for k, v in sorted(other.items(), key=lambda kv: -sum(kv[1])):
    v = np.array(v)
    print('%-60s n %5d median %.3f p90 %.3f max %.3f sum %.1f ms' % (
        k, len(v), np.median(v), np.percentile(v, 90), v.max(), v.sum()))
print('queues %d:' % len(queues))
for q, v in sorted(queues.items()):
    print('  queue %s: %s' % (q, dict(v)))
