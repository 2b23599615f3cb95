#!/usr/bin/env python3
"""Diagnostic (GPU box): one tile chip's sampled pixels through three paths -- the runner's rows
(transport encoding), Context.detect_batch of the whole chip (no encoding), the C oracle -- and the
magnitudes of the rows that differ.  python tools/diag_mag.py [--chips 0,1,2] [--config 3]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'lcmap-firebird_amd'), os.path.join(ROOT, 'oracle'), os.path.join(ROOT, 'tests'),
                os.path.join(ROOT, 'tools')]

import ccdgpu  # noqa: E402
import oracle_ctypes  # noqa: E402
import parity_util  # noqa: E402
import tile_parity as tp  # noqa: E402
from ccdc import runner  # noqa: E402
from ccdgpu import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--chips', default='0,1,2')
    ap.add_argument('--config', type=int, default=3)
    ap.add_argument('--encode', default='unread')
    args = ap.parse_args()
    chips = [int(c) for c in args.chips.split(',')]
    n = max(chips) + 1
    cfg = synth.config(args.config)
    src = synth.TileSource(cfg, batch_chips=6, pinned=True)
    sink = tp.SampleSink(100)
    xys = [(-1815585 + 3000 * (c // 50), 1064805 - 3000 * (c % 50)) for c in range(n)]
    enc = {'unread': True, 'lossless': 'lossless', 'none': False}[args.encode]
    runner.changedetection(xys, src, contexts=1, batch_chips=6, sink=sink, upload_depth=2, encode=enc)
    ctx = ccdgpu.Context()
    for c in chips:
        b = synth.TileSource(cfg, batch_chips=1, pinned=False)([c])
        d, s, q = b.chip(0)
        d, s, q = np.array(d), np.array(s), np.array(q)
        idx = tp.sample_pixels(c, 100)
        ora = oracle_ctypes.detect_batch(d, np.ascontiguousarray(s[:, idx]), np.ascontiguousarray(q[idx]), threads=8)
        n_, segs, ints, masks, floats, mr, notes = tp.compare_chip(c, sink.samples[c], ora, 100)
        print('chip', c, 'runner rows vs oracle: ints', ints, 'masks', masks, 'floats', floats, 'max rel', mr, flush=True)
        for t in notes[:6]:
            print('   ', t)
        got = ctx.detect_batch(d, np.ascontiguousarray(s[:, idx]), np.ascontiguousarray(q[idx]))
        probs, mrel = parity_util.compare(got, ora[1])
        print('chip', c, 'detect_batch (sample only) vs oracle:', len(probs), 'problems', probs[:4], flush=True)
        whole = ctx.detect_batch(d, s, q)
        sub_probs = []
        for j, p in enumerate(idx):
            a0, a1 = int(whole.seg_offsets[p]), int(whole.seg_offsets[p + 1])
            b0, b1 = int(ora[1].seg_offsets[j]), int(ora[1].seg_offsets[j + 1])
            ga, ra = whole.segments[a0:a1], ora[1].segments[b0:b1]
            if len(ga) != len(ra):
                sub_probs.append((j, 'count'))
                continue
            dm = np.abs(ga['magnitude'] - ra['magnitude'])
            if np.any(dm > 1e-6 * np.maximum(np.abs(ra['magnitude']), 1e-9)):
                sub_probs.append((j, 'mag'))
                if len(sub_probs) <= 3:
                    print('   sample', j, 'px', int(p), 'gpu mags', ga['magnitude'].tolist(), '\n   oracle mags', ra['magnitude'].tolist(),
                          '\n   change', ra['change_probability'].tolist(), 'bday', ra['break_day'].tolist(), 'eday', ra['end_day'].tolist())
        print('chip', c, 'detect_batch (whole chip) vs oracle on the sample:', len(sub_probs), sub_probs[:8], flush=True)


if __name__ == '__main__':
    main()
