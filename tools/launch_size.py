#!/usr/bin/env python3
"""Developer tool (GPU box): the detection kernel's own rate as a function of the launch size,
the CU reservation and the input form -- what separates the tile leg's in-kernel rate (8-chip
launches of transport-encoded batches on contexts that reserve CUs) from the resident leg's
(64-chip launches of raw batches).  One context, launches back to back, each launch's execution
window on the device clock (ccdgpu stats detect_ms_device) and its HIP-event duration.

    python tools/launch_size.py [--chips 64] [--config 3]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'lcmap-firebird_amd')]
import numpy as np  # noqa: E402
import bench  # noqa: E402
import ccdgpu  # noqa: E402
from ccdgpu import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--config', type=int, default=3)
ap.add_argument('--chips', type=int, default=64)
ap.add_argument('--reps', type=int, default=2)
a = ap.parse_args()
cfg = synth.config(a.config)
ids = bench.chip_ids(0, a.chips, 1, lambda c: bench.synth_nobs(cfg, c))
batch = bench.build_batch(cfg, ids)
chips = [batch.chip(c) for c in range(batch.n_chips)]
drop, strict = ccdgpu.unread_drop_bits(None)
out = {}


def run(tag, per, copy_cus, encode):
    ctx = ccdgpu.Context(0, copy_cus=copy_cus)
    groups = [chips[i:i + per] for i in range(0, len(chips), per)]
    if encode:
        bs = [ccdgpu.EncodedBatch.encode(g, threads=8, drop_bits=drop, strict_bits=strict) for g in groups]
    else:
        bs = [ccdgpu.ChipBatch.from_chips(g, pinned=True) for g in groups]
    # warm
    ctx.stage_slot_chips(0, bs[0])
    ctx.run_slot(0)
    dev, ev, px = [], [], 0
    for _ in range(a.reps):
        for b in bs:
            ctx.stage_slot_chips(0, b)
            ctx.synchronize()  # the upload is outside the kernel's window
            ctx.run_slot(0)
            st = ctx.stats()
            dev.append(st['detect_ms_device'])
            ev.append(st['detect_ms'])
            px += b.total_pixels
    ctx.close()
    rate = px / (sum(dev) * 1e-3)
    out[tag] = {'chips_per_launch': per, 'copy_cus': copy_cus, 'encoded': encode, 'launches': len(dev),
                'ms_device_median': float(np.median(dev)), 'ms_event_median': float(np.median(ev)),
                'px_per_s_device_clock': rate}
    print('%-12s %2d chips/launch cus %d enc %d: %.0f px/s (device clock), median %.2f ms' % (
        tag, per, copy_cus, encode, rate, float(np.median(dev))), flush=True)


run('c64_raw', 64, 0, False)
run('c8_raw', 8, 0, False)
run('c8_raw_cus8', 8, 8, False)
run('c8_enc_cus8', 8, 8, True)
run('c16_enc_cus8', 16, 8, True)
run('c32_enc_cus8', 32, 8, True)
run('c64_enc_cus8', 64, 8, True)
print(json.dumps(out))
