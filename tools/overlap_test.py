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
import numpy as np  # noqa: E402
import bench  # noqa: E402
import ccdgpu  # noqa: E402
from ccdgpu import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--config', type=int, default=3)
ap.add_argument('--per', type=int, default=8)
ap.add_argument('--launches', type=int, default=12)
ap.add_argument('--modes', default='run,fetch,upload')
ap.add_argument('--ns', default='1,4', help='context counts to run each mode with')
ap.add_argument('--pool-offset', type=int, default=0, help='--pool: first tile position of the batch')
ap.add_argument('--pool', action='store_true',
                help="the bench tile leg's chips (TileSource pool mode: date-shifted copies of GPU-generated chips, "
                     "positions 0..per-1) instead of the resident leg's")
a = ap.parse_args()
cfg = synth.config(a.config)
if a.pool:
    src = synth.TileSource(cfg, device=0, batch_chips=a.per, mode='pool', pool_chips=32)
    src.prepare()
    batch = ccdgpu.ChipBatch.from_chips([tuple(np.array(x) for x in v) for v in src.views(list(range(a.pool_offset, a.pool_offset + a.per)))])
    src.close()
else:
    ids = bench.chip_ids(0, 64, 1, lambda c: bench.synth_nobs(cfg, c))[::64 // a.per][:a.per]
    batch = bench.build_batch(cfg, ids)
out = {}


chips = [batch.chip(c) for c in range(batch.n_chips)]
drop, strict = ccdgpu.unread_drop_bits(None)
encs = [ccdgpu.EncodedBatch.encode(chips, threads=8, drop_bits=drop, strict_bits=strict) for _ in range(3)]
cx = [0] * batch.n_chips


KEPT = ('runenc', 'fetchenc', 'chain')  # slots staged once and kept (CCDGPU_KEEP_SLOTS=1): no uploads


def trial(tag, n_ctx, copy_cus, mode='run'):
    if mode in KEPT:
        os.environ['CCDGPU_KEEP_SLOTS'] = '1'
    ctxs = [ccdgpu.Context(0, copy_cus=copy_cus) for _ in range(n_ctx)]
    os.environ.pop('CCDGPU_KEEP_SLOTS', None)
    for c in ctxs:
        c.stage_chips(batch)
        c.run()
        if mode in KEPT:
            for s in range(3):
                c.stage_slot_chips(s, encs[s])
    for c in ctxs:
        c.synchronize()

    def go(c):
        bufs = ccdgpu.RowsBuffers()
        for i in range(a.launches):
            if mode in ('run', 'noise'):
                c.run()
            elif mode == 'fetch':
                c.run()
                c._keep = batch
                c.fetch_batch_rows_into(cx, cx, bufs)
            elif mode == 'runenc':  # encoded inputs read in place, no fetch
                c.run_slot(i % 3)
            elif mode == 'fetchenc':  # encoded inputs, detection then the separate rows fetch
                c.run_slot(i % 3)
                c.fetch_batch_rows_into(cx, cx, bufs)
            elif mode == 'chain':  # encoded inputs, the batch chain, no uploads
                c.run_slot_begin_rows(i % 3, cx, cx, bufs)
                c.run_slot_end_rows()
            elif mode == 'upload':  # upload an encoded batch (pinned, prepared), detect, fetch rows
                c.stage_slot_chips(i % 3, encs[i % 3])
                c.run_slot(i % 3)
                c.fetch_batch_rows_into(cx, cx, bufs)
            else:  # 'ahead': the runner's order -- the next upload staged while the detection runs
                if i == 0:
                    c.stage_slot_chips(0, encs[0])
                c.run_slot_begin_rows(i % 3, cx, cx, bufs)
                if i + 1 < a.launches:
                    c.stage_slot_chips((i + 1) % 3, encs[(i + 1) % 3])
                c.run_slot_end_rows()

    th = [threading.Thread(target=go, args=(c,)) for c in ctxs]
    stop = threading.Event()
    noise = None
    if mode == 'noise':
        # unrelated uploads at the tile's rate (one 8-chip encoded batch per ~28 ms) into a context
        # that never detects: the DMA traffic without any launch depending on it
        up = ccdgpu.Context(0, copy_cus=copy_cus)

        def upload():
            k = 0
            while not stop.is_set():
                up.stage_slot_chips(k % 3, encs[k % 3])
                k += 1
                time.sleep(0.028)
        noise = threading.Thread(target=upload)
        noise.start()
    t = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    el = time.perf_counter() - t
    if noise is not None:
        stop.set()
        noise.join()
        up.close()
    for c in ctxs:
        c.close()
    rate = n_ctx * a.launches * batch.total_pixels / el
    out[tag] = rate
    print('%-16s contexts %d copy_cus %d mode %s: %.0f px/s' % (tag, n_ctx, copy_cus, mode, rate), flush=True)


for mode in a.modes.split(','):
    for n in [int(x) for x in a.ns.split(',')]:
        trial('%s_n%d' % (mode, n), n, 8, mode)
print(json.dumps({'per': a.per, 'launches': a.launches, 'pool': a.pool, 'pool_offset': a.pool_offset, 'rates': out,
                  'GPU_MAX_HW_QUEUES': os.environ.get('GPU_MAX_HW_QUEUES')}))
