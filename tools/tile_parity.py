#!/usr/bin/env python3
"""Tile-scale parity (GPU box): the product tile driver ``ccdc.runner.changedetection``
(reference core.changedetection, ccdc/core.py:97-108) over a full tile of DISTINCT chips --
every tile position its own generated chip (ccdgpu.synth.TileSource: the device generator, the
same samples as the host generator) -- with a fixed stratified sample of every chip's pixels
checked against the C restatement oracle (oracle/libccdoracle.so) on the host, while the GPU runs.

Sample: ``--sample`` pixels per chip, one per image row band: pixel (row, col) with
row = k * 100 / sample and col = (37 k + 11 chip) mod 100, so every chip contributes pixels from
top to bottom and columns move between chips.  Compared per sampled pixel, from the device rows
the runner's sink receives (float32 segment rows, ccd_rows.hip) and the processing-mask bit words:
row count (= segment count, or the default row), start / end / break day, curve QA, change
probability, has_model, processing mask -- all bit-exact; magnitudes, RMSE, intercepts and
coefficients within 1e-6 relative of the oracle's float32-rounded values (plus one float32 ulp
for the double rounding).

    python tools/tile_parity.py [--chips 2500] [--sample 100] [--config 3] [--out FILE]
"""
import argparse
import json
import os
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'lcmap-firebird_amd'), os.path.join(ROOT, 'oracle'), os.path.join(ROOT, 'tests')]

import ccdgpu  # noqa: E402
import oracle_ctypes  # noqa: E402
import rows_util  # noqa: E402
from ccdc import runner  # noqa: E402
from ccdgpu import synth  # noqa: E402

TILE = 2500
RTOL = 1e-6
F32_ULP = 2.0 ** -23
INT_ROW_FIELDS = ('sday', 'eday', 'bday', 'curqa', 'has_model', 'chprob')
FLOAT_ROW_FIELDS = ('mag', 'rmse', 'intercept', 'coef')


def sample_pixels(pos, n):
    rows = [k * 100 // n for k in range(n)]
    return np.array([r * 100 + (37 * k + 11 * pos) % 100 for k, r in enumerate(rows)], dtype=np.int64)


class ParitySource(synth.TileSource):
    """TileSource that also hands every chip's sampled pixels to the oracle pool."""

    def __init__(self, cfg, pool, n_sample, **kw):
        super(ParitySource, self).__init__(cfg, **kw)
        self.pool = pool
        self.n_sample = n_sample
        self.futures = {}
        self._flock = threading.Lock()

    def __call__(self, positions):
        b = super(ParitySource, self).__call__(positions)
        for j, p in enumerate(positions):
            d, s, q = b.chip(j)
            idx = sample_pixels(p, self.n_sample)
            job = (np.array(d), np.ascontiguousarray(s[:, idx]), np.ascontiguousarray(q[idx]))
            with self._flock:
                self.futures[p] = self.pool.submit(lambda a: oracle_ctypes.detect_batch(*a, threads=1), job)
        return b


class SampleSink(runner.SummarySink):
    """Keeps the sampled pixels' rows and mask words of every chip (and the usual summaries)."""

    def __init__(self, n_sample):
        super(SampleSink, self).__init__(digest=True)
        self.n_sample = n_sample
        self.samples = {}

    def __call__(self, pos, cx, cy, dates, row_offsets, rows, mask_bits):
        super(SampleSink, self).__call__(pos, cx, cy, dates, row_offsets, rows, mask_bits)
        idx = sample_pixels(pos, self.n_sample)
        per = [np.array(rows[int(row_offsets[p]):int(row_offsets[p + 1])]) for p in idx]
        self.samples[int(pos)] = (per, np.array(mask_bits[idx]), int(cx), int(cy), int(dates.shape[0]))


def compare_chip(pos, dev, ora, n_sample):
    """-> (pixels, segments, int mismatches, mask mismatches, float mismatches, max rel, notes)"""
    per, bits, cx, cy, n_obs = dev
    rc, u = ora
    notes = []
    if rc != 0:
        return n_sample, 0, n_sample, 0, 0, 0.0, ['oracle rc %d' % rc]
    off, rows = rows_util.rows_from_result(u, cx, cy)
    words = bits.shape[1]
    ref_bits = rows_util.mask_words(u.mask, words)
    ints = masks = floats = segs = 0
    max_rel = 0.0
    for j in range(n_sample):
        g = per[j]
        r = rows[int(off[j]):int(off[j + 1])]
        segs += len(r)
        if not np.array_equal(bits[j], ref_bits[j]):
            masks += 1
            notes.append('chip %d sample %d: processing mask differs' % (pos, j))
        if len(g) != len(r):
            ints += 1
            notes.append('chip %d sample %d: %d rows vs oracle %d: %s vs %s' % (
                pos, j, len(g), len(r), g[['sday', 'eday', 'bday']].tolist(), r[['sday', 'eday', 'bday']].tolist()))
            continue
        for f in INT_ROW_FIELDS:
            bad = g[f] != r[f]
            if np.any(bad):
                ints += int(np.count_nonzero(bad))
                notes.append('chip %d sample %d: %s %s vs %s' % (pos, j, f, g[f].tolist(), r[f].tolist()))
        for f in FLOAT_ROW_FIELDS:
            a, b = g[f].astype(np.float64), r[f].astype(np.float64)
            diff = np.abs(a - b)
            scale = np.maximum(np.abs(a), np.abs(b))
            bad = diff > (RTOL + 2 * F32_ULP) * scale + 1e-9
            with np.errstate(divide='ignore', invalid='ignore'):
                rel = np.where(scale > 0, diff / scale, 0.0)
            if rel.size:
                max_rel = max(max_rel, float(np.max(rel)))
            if np.any(bad):
                floats += int(np.count_nonzero(bad))
                notes.append('chip %d sample %d: %s max rel %.3e' % (pos, j, f, float(np.max(rel))))
    return n_sample, segs, ints, masks, floats, max_rel, notes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--chips', type=int, default=TILE)
    ap.add_argument('--sample', type=int, default=100)
    ap.add_argument('--config', type=int, default=3)
    ap.add_argument('--batch', type=int, default=8)
    ap.add_argument('--offset', type=int, default=0,
                    help='generator chip of position 0 (2500: the next tile\'s chips, other seeds and cadences)')
    ap.add_argument('--oracle-threads', type=int, default=int(os.environ.get('OMP_NUM_THREADS', '16') or 16) - 1)
    ap.add_argument('--out', default=os.path.join(ROOT, 'gpurun_out', 'tile_parity.json'))
    ap.add_argument('--encode', choices=('unread', 'lossless', 'none'), default='unread', help='upload of the chips (the runner\'s default: unread)')
    ap.add_argument('--cpu-dry-run', action='store_true',
                    help='plumbing check without a GPU: host generator, oracle-backed contexts (tests/rows_util)')
    args = ap.parse_args()
    cfg = synth.config(args.config)
    pool = ThreadPoolExecutor(max(1, args.oracle_threads))
    factory = None
    if args.cpu_dry_run:
        class HostGen(object):
            def batch(self, cfg, ids, n_pix=10000, pix0=0, out=None):
                for j, c in enumerate(ids):
                    synth.chip(cfg, c, pix0, n_pix, out=out.chip(j))
                return out

            def dates(self, cfg, c):
                return synth.dates(cfg, c)

            def close(self):
                pass
        synth.TileSource._gen = lambda self: HostGen()
        factory = lambda dev: rows_util.OracleContext(dev, threads=4)
    src = ParitySource(cfg, pool, args.sample, batch_chips=args.batch, pinned=not args.cpu_dry_run,
                       chip_of=lambda pos: int(pos) + args.offset)
    sink = SampleSink(args.sample)
    xys = [(-1815585 + 3000 * (c // 50), 1064805 - 3000 * (c % 50)) for c in range(args.chips)]
    t = time.perf_counter()
    enc = {'unread': True, 'lossless': 'lossless', 'none': False}[args.encode]
    res = runner.changedetection(xys, src, contexts=2, batch_chips=args.batch, sink=sink, upload_depth=2,
                                 context_factory=factory, encode=enc)
    gpu_s = time.perf_counter() - t
    print('tile of %d chips detected in %.1f s; waiting for the oracle' % (args.chips, gpu_s), flush=True)
    tot = {'pixels': 0, 'segments': 0, 'int_mismatches': 0, 'mask_mismatches': 0, 'float_mismatches': 0}
    max_rel = 0.0
    notes = []
    bad_chips = []
    last = time.perf_counter()
    for k, p in enumerate(sorted(src.futures)):
        ora = src.futures[p].result()
        n, segs, ints, masks, floats, mr, nt = compare_chip(p, sink.samples[p], ora, args.sample)
        tot['pixels'] += n
        tot['segments'] += segs
        tot['int_mismatches'] += ints
        tot['mask_mismatches'] += masks
        tot['float_mismatches'] += floats
        max_rel = max(max_rel, mr)
        if ints or masks or floats:
            bad_chips.append(p)
            notes += nt[:3]
        if time.perf_counter() - last > 30:
            print('compared %d / %d chips' % (k + 1, len(src.futures)), flush=True)
            last = time.perf_counter()
    total_s = time.perf_counter() - t
    mix = {}
    for c in res['chips']:
        mix[c['n_obs']] = mix.get(c['n_obs'], 0) + 1
    out = {
        'what': 'tile parity: ccdc.runner.changedetection over %d distinct generated chips (config %d, generator chips '
                '%d ..), a stratified sample of %d pixels per chip vs the C restatement oracle' % (
                    args.chips, args.config, args.offset, args.sample),
        'chips': len(res['chips']), 'distinct_chip_ids': len(set(src.futures)), 'n_obs_mix': mix,
        'tile_pixels': sum(c['n_pix'] for c in res['chips']), 'tile_rows': sum(c['rows'] for c in res['chips']),
        'sampled_pixels': tot['pixels'], 'sampled_rows': tot['segments'],
        'int_mismatches': tot['int_mismatches'], 'mask_mismatches': tot['mask_mismatches'],
        'float_mismatches': tot['float_mismatches'], 'max_float_rel_diff': max_rel,
        'chips_with_mismatches': bad_chips[:50], 'first_mismatches': notes[:20],
        'detect_seconds': gpu_s, 'total_seconds': total_s, 'generate_seconds': src.generate_seconds,
        'oracle_threads': args.oracle_threads,
        'upload': {'unread': 'transport encoding, unread setting (band values of fill/cloud/shadow observations not sent)',
                   'lossless': 'transport encoding, lossless setting', 'none': 'raw'}[args.encode],
        'compare': 'rows and mask words: row count, sday/eday/bday, curqa, has_model, chprob, processing mask bit-exact; '
                   'mag/rmse/intercept/coef within 1e-6 relative + 2 float32 ulp of the oracle rows',
        'chip_digests_sha1': __import__('hashlib').sha1(''.join(c['digest'] for c in res['chips']).encode()).hexdigest(),
    }
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, 'w') as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k not in ('first_mismatches', 'chips_with_mismatches')}), flush=True)
    src.close()
    pool.shutdown()
    return 0 if not (tot['int_mismatches'] or tot['mask_mismatches'] or tot['float_mismatches']) else 1


if __name__ == '__main__':
    sys.exit(main())
