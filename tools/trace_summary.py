#!/usr/bin/env python3
"""Developer tool: per-kernel duration percentiles of a rocprofv3 --kernel-trace rocpd database
over the last `seconds` of the trace (bench tile JSON), plus memory-copy percentiles by direction
and size class.  usage: trace_summary.py <run_results.db> <tile.json>"""
import json
import sqlite3
import sys


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))] if v else None


def main():
    db, js = sys.argv[1], sys.argv[2]
    secs = float(json.load(open(js))['tile']['seconds'])
    c = sqlite3.connect(db)
    ks = list(c.execute('select name, start, end from kernels'))
    end = max(e for _, _, e in ks)
    lo = end - int(secs * 1e9)
    agg = {}
    for n, a, b in ks:
        if a < lo:
            continue
        k = n.replace('(anonymous namespace)::', '').split('(')[0][:60]
        agg.setdefault(k, []).append((b - a) / 1e6)
    out = {'kernels': {k: {'n': len(v), 'p50_ms': pct(v, .5), 'p90_ms': pct(v, .9), 'p99_ms': pct(v, .99), 'max_ms': max(v),
                           'sum_ms': round(sum(v), 1)} for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))}}
    cols = [r[1] for r in c.execute('pragma table_info(memory_copies)')]
    ci = {k: i for i, k in enumerate(cols)}
    cp = {}
    for r in c.execute('select * from memory_copies'):
        if r[ci['start']] < lo:
            continue
        d = 'd2h' if 'DEVICE_TO_HOST' in str(r[ci['name']]) else 'h2d' if 'HOST_TO_DEVICE' in str(r[ci['name']]) else 'other'
        sz = r[ci['size']]
        cls = 'small' if sz < 65536 else 'mid' if sz < (8 << 20) else 'big'
        cp.setdefault(d + '_' + cls, []).append(((r[ci['end']] - r[ci['start']]) / 1e6, sz))
    out['copies'] = {k: {'n': len(v), 'p50_ms': pct([x for x, _ in v], .5), 'p90_ms': pct([x for x, _ in v], .9),
                         'max_ms': max(x for x, _ in v), 'sum_ms': round(sum(x for x, _ in v), 1),
                         'bytes_p50': pct([s for _, s in v], .5)} for k, v in sorted(cp.items())}
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
