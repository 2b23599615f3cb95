#!/usr/bin/env python3
"""Timeline of a traced tile run (rocprofv3 --kernel-trace --memory-copy-trace, rocpd database):
over the timed window (the last `seconds` of the trace, from bench.py's tile JSON) the fraction
of wall time covered by at least one detection kernel, the time fractions with 0, 1, 2, ...
detection launches in flight, by at least one host-to-device copy, by
both, and by neither; the H2D bytes and rate; the detection kernels' summed durations; and the
upload decode kernel's durations (median, max).

usage: tile_timeline.py <run_results.db> <tile.json>"""
import json
import sqlite3
import sys


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def clip(iv, lo, hi):
    return [(max(a, lo), min(b, hi)) for a, b in iv if b > lo and a < hi]


def length(iv):
    return sum(b - a for a, b in iv)


def intersect(x, y):
    out, i, j = [], 0, 0
    while i < len(x) and j < len(y):
        a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
        if a < b:
            out.append((a, b))
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return out


def main():
    db, js = sys.argv[1], sys.argv[2]
    secs = float(json.load(open(js))['tile']['seconds'])
    c = sqlite3.connect(db)
    det = [(s, e) for n, s, e in c.execute('select name, start, end from kernels') if 'ccd_detect' in n]
    cols = [r[1] for r in c.execute('pragma table_info(memory_copies)')]
    rows = list(c.execute('select * from memory_copies'))
    ci = {k: i for i, k in enumerate(cols)}
    h2d = []
    nbytes = 0
    for r in rows:
        kind = str(r[ci['name']]) if 'name' in ci else ''
        if 'HOST_TO_DEVICE' in kind.upper() or 'HTOD' in kind.upper().replace('_', ''):
            h2d.append((r[ci['start']], r[ci['end']], r[ci['size']] if 'size' in ci else 0))
    end = max(max(e for _, e in det), max((e for _, e, _ in h2d), default=0))
    lo, hi = end - int(secs * 1e9), end
    d = clip(union(det), lo, hi)
    h = clip(union([(a, b) for a, b, _ in h2d]), lo, hi)
    nbytes = sum(n for a, b, n in h2d if a >= lo)
    dec = [e - s for n, s, e in c.execute('select name, start, end from kernels') if 'decode_enc' in n and s >= lo]
    both = intersect(d, h)
    wall = hi - lo
    # how many detection launches are in flight at once (each is one context's batch): the time
    # fraction with 0, 1, 2, ... of them -- with one alone the GPU is draining its tail
    ev = sorted([(max(a, lo), 1) for a, b in det if b > lo and a < hi] + [(min(b, hi), -1) for a, b in det if b > lo and a < hi])
    conc, cur, last = {}, 0, lo
    for t, dlt in ev:
        conc[cur] = conc.get(cur, 0) + (t - last)
        cur += dlt
        last = t
    conc[cur] = conc.get(cur, 0) + (hi - last)
    out = {'window_s': wall / 1e9, 'detect_covered': length(d) / wall, 'h2d_covered': length(h) / wall,
           'both': length(both) / wall, 'neither': 1 - (length(d) + length(h) - length(both)) / wall,
           'h2d_bytes': nbytes, 'h2d_gbs_over_window': nbytes / wall, 'h2d_gbs_while_copying': nbytes / max(1, length(h)),
           'detect_dispatches': sum(1 for a, b in det if a >= lo),
           'detect_kernel_seconds_summed': sum(b - a for a, b in det if a >= lo) / 1e9,
           'decode_dispatches': len(dec), 'decode_ms_median': (sorted(dec)[len(dec) // 2] / 1e6) if dec else None,
           'decode_ms_max': (max(dec) / 1e6) if dec else None,
           'detections_in_flight_time_fraction': {str(k): round(v / wall, 4) for k, v in sorted(conc.items())},
           'detect_ms_median': sorted(b - a for a, b in det if a >= lo)[len([1 for a, b in det if a >= lo]) // 2] / 1e6,
           'copy_kinds': sorted({str(r[ci['name']]) for r in rows}) if 'name' in ci else cols}
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
