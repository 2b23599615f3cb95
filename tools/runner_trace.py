#!/usr/bin/env python3
"""Developer tool: per-worker pipeline phases of a tile run with CCDC_RUNNER_TRACE=1 (bench.py's
tile.runner_trace_rank0): per batch the launch -> detection-done time, the done -> next launch
gap (finish + row fetch + sink + staging), and how often a worker had no staged batch to launch.
usage: runner_trace.py <bench.json>"""
import json
import sys

d = json.load(open(sys.argv[1]))
tr = d['tile']['runner_trace_rank0']


def pct(v, q):
    v = sorted(v)
    return round(v[min(len(v) - 1, int(q * len(v)))] * 1e3, 2) if v else None


run_ms, post_ms, fetch_ms, wait_ms, stage_to_launch = [], [], [], [], []
for w in tr:
    runs = [x for x in w if x[0] == 'run']
    stages = {x[1]: x[2] for x in w if x[0] == 'stage'}
    for i, (_, p, t2, te, t3, t4, t5) in enumerate(runs):
        run_ms.append(t3 - t2)
        fetch_ms.append(t4 - t3)
        wait_ms.append(t3 - te)
        if p in stages:
            stage_to_launch.append(t2 - stages[p])
        if i + 1 < len(runs):
            post_ms.append(runs[i + 1][2] - t3)
out = {k: {'p10': pct(v, .1), 'p50': pct(v, .5), 'p90': pct(v, .9), 'sum_s': round(sum(v), 2), 'n': len(v)}
       for k, v in (('launch_to_done_ms', run_ms), ('done_to_next_launch_ms', post_ms), ('row_fetch_ms', fetch_ms),
                    ('staged_to_launch_ms', stage_to_launch), ('end_wait_ms', wait_ms))}
out['value'] = d['value']
print(json.dumps(out, indent=1))
