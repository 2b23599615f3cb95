#!/usr/bin/env python3
"""Developer tool (GPU box): ccdc.pyccd.detect_partition end to end on one Python worker -- merlin-
style per-pixel records (Python lists) of C3 / C5 chips in, the reference's row dicts out --
pixels/s and the split between packing, device and formatting."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'lcmap-firebird_amd')]
import ccd  # noqa: E402
from ccdc import pyccd, timeseries  # noqa: E402
from ccdgpu import synth  # noqa: E402

for cfgn, chip, n_pix in ((3, 0, 4000), (5, 3, 2000)):
    d, s, q = synth.chip(synth.config(cfgn), chip, 0, n_pix)
    dl = [int(x) for x in d]
    keys = timeseries.chip_keys(-1815585, 1064805, n_pix)
    recs = []
    for p in range(n_pix):
        rec = {'dates': dl, 'qas': q[p].tolist()}
        for b, kw in enumerate(ccd.BAND_KWARGS):
            rec[kw] = s[b, p].tolist()
        recs.append((keys[p], rec))
    pyccd.detect_partition(recs[:64])  # warm: context, library
    t = time.perf_counter()
    rows = pyccd.detect_partition(recs)
    el = time.perf_counter() - t
    print('C%d: %d pixels, %d rows in %.2f s: %.0f px/s per worker' % (cfgn, n_pix, len(rows), el, n_pix / el), flush=True)
