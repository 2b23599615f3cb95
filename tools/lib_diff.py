#!/usr/bin/env python3
"""Developer tool (GPU box): byte comparison of two detection libraries' results on the same
chips (segments, masks, procedures in float64, not the float32 rows) -- for kernel changes
meant to leave every output bit as it was.

    python tools/lib_diff.py lib/libccdgpu.so lib/other.so [--chips 3:0,3:3,5:1,2:0 --pixels 4000]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'lcmap-firebird_amd')]
import numpy as np  # noqa: E402
import ccdgpu  # noqa: E402
from ccdgpu import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('libs', nargs=2)
ap.add_argument('--chips', default='3:0,3:3,5:1,5:4,2:0,4:1')
ap.add_argument('--pixels', type=int, default=4000)
a = ap.parse_args()
cases = [tuple(int(x) for x in c.split(':')) for c in a.chips.split(',')]
inputs = [synth.chip(synth.config(cfg), chip, 0, a.pixels) for cfg, chip in cases]
outs = []
for path in a.libs:
    ccdgpu._lib = None
    ccdgpu.LIB_PATH = path if os.path.isabs(path) else os.path.join(ROOT, 'lcmap-firebird_amd', path)
    ctx = ccdgpu.Context(0)
    got = []
    for d, s, q in inputs:
        r = ctx.detect_batch(d, s, q)
        got.append({k: np.ascontiguousarray(getattr(r, k)) for k in ('segments', 'seg_offsets', 'mask', 'procedure', 'probs')})
    ctx.close()
    outs.append(got)
bad = 0
for (cfg, chip), x, y in zip(cases, outs[0], outs[1]):
    for k in x:
        same = x[k].shape == y[k].shape and x[k].tobytes() == y[k].tobytes()
        if not same:
            bad += 1
            print('C%d chip %d: %s differs' % (cfg, chip, k))
    print('C%d chip %d: %d pixels, %d segments compared' % (cfg, chip, a.pixels, x['segments'].shape[0]), flush=True)
print('lib_diff: %s' % ('IDENTICAL' if bad == 0 else '%d arrays differ' % bad))
sys.exit(1 if bad else 0)
