#!/usr/bin/env python3
"""How many pixels' outputs depend on the argsort tie rule: the C restatement
oracle run twice over the same pixels -- numpy quicksort tie order (the pinned reference's,
ARGSORT 'quicksort', the default since round 6) and the stable rule of rounds 1-5 -- and the
pixels compared under the suite's parity bar (tests/parity_util.py).  CPU only.

Pixels: the tile-parity sample (tools/tile_parity.py: ``--sample`` stratified pixels of each of
the ``--chips`` tile chips of config 3, both cadences) plus ``--c5-chips`` change-dense chips of
config 5 (``--c5-sample`` stratified pixels each).  Also reports the oracle's closest-DOY counters
(ccdoracle_argsort_stats): selections over > 24 fit observations, those with ties across the 24th
position, those where the stable rule takes another set, argsort parts past numpy 1.17's
introsort depth limit.

    python tools/argsort_exposure.py [--chips 2500] [--sample 100] [--c5-chips 16] [--out FILE]
"""
import argparse
import ctypes
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'lcmap-firebird_amd'), os.path.join(ROOT, 'oracle'), os.path.join(ROOT, 'tests')]

import oracle_ctypes  # noqa: E402
import parity_util  # noqa: E402
from ccdgpu import synth  # noqa: E402


def sample_pixels(pos, n):
    rows = [k * 100 // n for k in range(n)]
    return np.array([r * 100 + (37 * k + 11 * pos) % 100 for k, r in enumerate(rows)], dtype=np.int64)


def pixels(cfg, chip, idx):
    d = synth.dates(cfg, chip)
    n = d.shape[0]
    s = np.empty((7, len(idx), n), np.int16)
    q = np.empty((len(idx), n), np.uint16)
    for j, px in enumerate(idx):
        _, ss, qq = synth.chip(cfg, chip, int(px), 1, chip_dates=d)
        s[:, j], q[j] = ss[:, 0], qq[0]
    return d, s, q


def stats(reset):
    L = oracle_ctypes.lib()
    L.ccdoracle_argsort_stats.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    out = np.zeros(4, np.int64)
    L.ccdoracle_argsort_stats(out.ctypes.data, int(reset))
    return out


def run(cfg_no, chips, n_sample, threads):
    cfg = synth.config(cfg_no)

    def one(chip):
        d, s, q = pixels(cfg, chip, sample_pixels(chip, n_sample))
        rq, gq = oracle_ctypes.detect_batch(d, s, q, params=None, threads=1)
        rs, gs = oracle_ctypes.detect_batch(d, s, q, params={'ARGSORT': 'stable'}, threads=1)
        assert rq == 0 and rs == 0
        bad = []
        for px in range(q.shape[0]):
            sub = lambda u: _pixel(u, px)
            probs, _ = parity_util.compare(sub(gq), sub(gs))
            if probs:
                bad.append((chip, int(px), probs[0]))
        return q.shape[0], int(gq.seg_offsets[-1]), bad

    stats(True)
    t0 = time.time()
    n_px = n_seg = 0
    diffs = []
    with ThreadPoolExecutor(threads) as ex:
        for k, (npx, nseg, bad) in enumerate(ex.map(one, chips)):
            n_px += npx
            n_seg += nseg
            diffs += bad
            if k % 100 == 99:
                print('config %d: %d chips, %d px, %d differ, %.0f s' % (cfg_no, k + 1, n_px, len(diffs), time.time() - t0),
                      flush=True)
    st = stats(True)
    return {'config': cfg_no, 'chips': len(chips), 'pixels': n_px, 'segments_quicksort': n_seg,
            'pixels_differing': len(diffs), 'examples': [list(map(str, d)) for d in diffs[:20]],
            'closest_selections_over_24': int(st[0]), 'with_ties_across_24th': int(st[1]),
            'stable_takes_another_set': int(st[2]), 'introsort_depth_limit_parts': int(st[3]),
            'seconds': round(time.time() - t0, 1)}


class _pixel(object):
    """one pixel of an abi.Unpacked as a 1-pixel Unpacked-like view (for parity_util.compare)"""

    def __init__(self, u, px):
        a, b = u.seg_offsets[px], u.seg_offsets[px + 1]
        self.n_pix, self.n_obs = 1, u.n_obs
        self.sorted_dates, self.sort_index = u.sorted_dates, u.sort_index
        self.procedure = u.procedure[px:px + 1]
        self.mask = u.mask[px:px + 1]
        self.seg_offsets = np.array([0, b - a])
        self.segments = u.segments[a:b]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--chips', type=int, default=2500)
    ap.add_argument('--sample', type=int, default=100)
    ap.add_argument('--c5-chips', type=int, default=16)
    ap.add_argument('--c5-sample', type=int, default=500)
    ap.add_argument('--threads', type=int, default=os.cpu_count() or 8)
    ap.add_argument('--out', default=os.path.join(ROOT, 'profiles', 'r06', 'argsort_exposure.json'))
    a = ap.parse_args()
    res = {'what': 'pixels whose C-oracle outputs differ between the numpy-quicksort and the stable argsort '
                   'tie rule (parity bar of tests/parity_util.py)', 'legs': []}
    res['legs'].append(run(3, list(range(a.chips)), a.sample, a.threads))
    res['legs'].append(run(5, list(range(a.c5_chips)), a.c5_sample, a.threads))
    print(json.dumps(res, indent=1))
    with open(a.out, 'w') as f:
        json.dump(res, f, indent=1)


if __name__ == '__main__':
    main()
