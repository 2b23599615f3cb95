#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 --kernel-trace --stats run written as a rocpd SQLite database
(ROCm 7's default output format): calls, total / average / median / min / max duration in ns, as
CSV (the columns of rocprofv3's kernel_stats.csv plus the median).

The median is printed beside the average because the bench overlaps two contexts: a dispatch
queued behind the other context's running launch is timed by the profiler from its own dispatch,
so one duration per overlap covers both launches (e.g. 447 ms among 226 ms ones).

usage: rocpd_stats.py <run_results.db> [out.csv]"""
import csv
import sqlite3
import statistics
import sys


def main():
    db = sys.argv[1]
    c = sqlite3.connect(db)
    per = {}
    for name, start, end in c.execute('select name, start, end from kernels'):
        per.setdefault(name, []).append(float(end - start))
    rows = []
    for name, d in per.items():
        rows.append({'Name': name[:160], 'Calls': len(d), 'TotalDurationNs': sum(d), 'AverageNs': sum(d) / len(d),
                     'MedianNs': statistics.median(d), 'MinNs': min(d), 'MaxNs': max(d)})
    rows.sort(key=lambda r: -r['TotalDurationNs'])
    out = open(sys.argv[2], 'w', newline='') if len(sys.argv) > 2 else sys.stdout
    w = csv.DictWriter(out, fieldnames=list(rows[0].keys()))
    w.writeheader()
    for r in rows:
        w.writerow(r)


if __name__ == '__main__':
    main()
