#!/usr/bin/env python3
"""Developer tool (GPU box): do detection launches of different contexts overlap (the next
launch's waves filling the previous one's tail)?  Every context stages the same 8-chip batch once;
N threads run K launches each concurrently; the aggregate rate against one context alone shows
whether a launch's tail is filled by another context's launch.

    python tools/overlap_test.py [--per 8] [--launches 12]
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'lcmap-firebird_amd')]
import bench  # noqa: E402
import ccdgpu  # noqa: E402
from ccdgpu import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--config', type=int, default=3)
ap.add_argument('--per', type=int, default=8)
ap.add_argument('--launches', type=int, default=12)
a = ap.parse_args()
cfg = synth.config(a.config)
ids = bench.chip_ids(0, 64, 1, lambda c: bench.synth_nobs(cfg, c))[::64 // a.per][:a.per]
batch = bench.build_batch(cfg, ids)
out = {}


def trial(tag, n_ctx, copy_cus):
    ctxs = [ccdgpu.Context(0, copy_cus=copy_cus) for _ in range(n_ctx)]
    for c in ctxs:
        c.stage_chips(batch)
        c.run()
    for c in ctxs:
        c.synchronize()

    def go(c):
        for _ in range(a.launches):
            c.run()

    th = [threading.Thread(target=go, args=(c,)) for c in ctxs]
    t = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    el = time.perf_counter() - t
    for c in ctxs:
        c.close()
    rate = n_ctx * a.launches * batch.total_pixels / el
    out[tag] = rate
    print('%-16s contexts %d copy_cus %d: %.0f px/s' % (tag, n_ctx, copy_cus, rate), flush=True)


for cus in (0, 8):
    for n in (1, 2, 4):
        trial('n%d_cus%d' % (n, cus), n, cus)
print(json.dumps({'per': a.per, 'launches': a.launches, 'rates': out,
                  'GPU_MAX_HW_QUEUES': os.environ.get('GPU_MAX_HW_QUEUES')}))
