#!/usr/bin/env python3
"""Developer tool (GPU box): resident-rate A/B of kernel libraries on ONE generated batch, all in
one process (the batch is generated once; each library is loaded in turn), rounds interleaved so
drift on the box hits every library alike.

    python tools/ab_resident.py --config 3 --chips 64 --steps 8 --rounds 2 lib/libccdgpu.so lib/exp/x.so ...
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'lcmap-firebird_amd')]
import bench  # noqa: E402
import ccdgpu  # noqa: E402
from ccdgpu import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--config', type=int, default=3)
ap.add_argument('--chips', type=int, default=64)
ap.add_argument('--steps', type=int, default=8)
ap.add_argument('--warmup', type=int, default=2)
ap.add_argument('--rounds', type=int, default=2)
ap.add_argument('--contexts', type=int, default=2)
ap.add_argument('libs', nargs='+')
a = ap.parse_args()
cfg = synth.config(a.config)
ids = bench.chip_ids(0, a.chips, 1, lambda c: bench.synth_nobs(cfg, c))
batch = bench.build_batch(cfg, ids)
res = {}
for r in range(a.rounds):
    for spec in a.libs:
        # "lib.so:w3" runs the library's 3-waves/SIMD kernel (CCDGPU_KERNEL, read at context creation)
        path, _, variant = spec.partition(':')
        if variant:
            os.environ['CCDGPU_KERNEL'] = variant
        else:
            os.environ.pop('CCDGPU_KERNEL', None)  # the library's default kernel
        ccdgpu._lib = None
        ccdgpu.LIB_PATH = path if os.path.isabs(path) else os.path.join(ROOT, 'lcmap-firebird_amd', path)
        ns = argparse.Namespace(chips=a.chips, contexts=a.contexts, warmup=a.warmup, steps=a.steps, config=a.config, roofline_launches=1)
        out = bench.resident_leg(ns, cfg, 0, 1, 0, None, batch=batch)
        rate = out['value']
        res.setdefault(spec, []).append({'value': rate, 'frac': out['roofline']['frac'],
                                         'kernel_ms': out['roofline']['kernel_ms_per_launch']})
        print('C%d %-40s round %d  %.0f px/s  frac %.4f  kernel %.1f ms' % (
            a.config, os.path.basename(spec), r, rate, out['roofline']['frac'], out['roofline']['kernel_ms_per_launch']),
            flush=True)
print(json.dumps({'config': a.config, 'chips': a.chips, 'workload_key': out['workload_key'], 'results': res}))
