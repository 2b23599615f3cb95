"""Chip packer timing: ccd_unpack_b64 on chipmunk text of C3-shaped chips (10^4 pixels x 1421
dates), median of 10 device-timed launches, for 1 and 8 chips per launch.  Run once per form
(CCDGPU_UNPACK_V1=1 selected the round-5 form while both existed)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'lcmap-firebird_amd'))
import ccdgpu  # noqa: E402
from ccdc import chipmunk  # noqa: E402

rng = np.random.default_rng(0)
n_pix, n_obs = 10000, 1421
dates = np.sort(rng.choice(np.arange(724000, 738000), n_obs, replace=False))[::-1].astype(np.int64)
S = rng.integers(-2000, 9000, size=(7, n_pix, n_obs), dtype=np.int16)
Q = rng.choice(np.array([1, 66, 68, 72, 80, 96, 112], np.uint16), size=(n_pix, n_obs))
ctx = ccdgpu.Context(0)
out = {'form': 'v1' if os.environ.get('CCDGPU_UNPACK_V1') == '1' else 'v2'}
for nc in (1, 8):
    locs = []
    for c in range(nc):
        chips = chipmunk.chip_response(3000 * c, 0, dates, np.roll(S, c, axis=1), np.roll(Q, c, axis=0))
        locs.append(chipmunk.group(chips)[(3000 * c, 0)])
    d, text, offsets = chipmunk.pack_text(locs)
    ctx.stage_chipmunk(d, text, offsets, n_pix)
    ks = [ctx.stage_chipmunk(d, text, offsets, n_pix) for _ in range(10)]
    k = float(np.median(ks))
    moved = len(text) + 2 * 8 * n_pix * n_obs * nc
    out[f'chips{nc}'] = {'kernel_ms': round(k * 1e3, 4), 'bytes': moved, 'gbs': round(moved / k / 1e9, 1)}
    print(json.dumps(out), flush=True)
ctx.close()
