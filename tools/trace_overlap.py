#!/usr/bin/env python3
"""Developer tool: for the short kernels of a traced tile run (every kernel but the detection),
their duration split by whether a large host-to-device copy (> 8 MiB: a batch upload) was in
flight when they started.  usage: trace_overlap.py <run_results.db> <tile.json>"""
import bisect
import json
import sqlite3
import sys


def pct(v, q):
    v = sorted(v)
    return round(v[min(len(v) - 1, int(q * len(v)))], 3) if v else None


db, js = sys.argv[1], sys.argv[2]
secs = float(json.load(open(js))['tile']['seconds'])
c = sqlite3.connect(db)
ks = list(c.execute('select name, start, end from kernels'))
end = max(e for _, _, e in ks)
lo = end - int(secs * 1e9)
cols = [r[1] for r in c.execute('pragma table_info(memory_copies)')]
ci = {k: i for i, k in enumerate(cols)}
up = sorted((r[ci['start']], r[ci['end']]) for r in c.execute('select * from memory_copies')
            if 'HOST_TO_DEVICE' in str(r[ci['name']]) and r[ci['size']] > (8 << 20))
starts = [a for a, _ in up]


def during_upload(t):
    i = bisect.bisect_right(starts, t) - 1
    return i >= 0 and up[i][1] > t


out = {}
for n, a, b in ks:
    if a < lo or 'ccd_detect' in n:
        continue
    k = n.replace('(anonymous namespace)::', '').split('(')[0][:40]
    out.setdefault(k, {'up': [], 'idle': []})['up' if during_upload(a) else 'idle'].append((b - a) / 1e6)
print(json.dumps({k: {w: {'n': len(v[w]), 'p50': pct(v[w], .5), 'p90': pct(v[w], .9), 'sum': round(sum(v[w]), 1)}
                      for w in ('up', 'idle')} for k, v in out.items()}, indent=1))
