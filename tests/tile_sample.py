"""Sampled-pixel parity of a tile run (ccdc.runner.changedetection) against the C oracle -- TEST
INFRASTRUCTURE: used by tests/test_gpu_tile.py and, after its timed region, by bench.py's tile
leg (the ``parity_sample`` it reports).  A ``PixelSampleSink`` keeps, for every chip the runner
hands over, the device-packed rows and processing-mask words of a few chosen pixels; ``check``
re-detects those pixels from their raw inputs with oracle/libccdoracle.so (reference semantics of
pyccd ccd.detect, ccdc/pyccd.py:168) and compares row for row: integer fields (coordinates, days,
curve QA, model flag), the row count and the mask bit for bit, float fields within 1e-6
relative."""
import os
import sys
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_HERE)
for _p in (os.path.join(_ROOT, 'oracle'), os.path.join(_ROOT, 'lcmap-firebird_amd'), _HERE):
    if _p not in sys.path:
        sys.path.insert(0, _p)

INT_FIELDS = ('px', 'py', 'sday', 'eday', 'bday', 'curqa', 'has_model')
FLOAT_FIELDS = ('chprob', 'mag', 'rmse', 'intercept', 'coef')


class PixelSampleSink(object):
    """Sink wrapper: ``pixels_of(pos)`` -> pixel indices of the chip at tile position ``pos``
    whose rows and mask words are kept (copies); every call is passed on to ``inner`` (default a
    SummarySink without digests, whose ``chips`` the runner gathers)."""

    def __init__(self, pixels_of, inner=None):
        from ccdc import runner
        self.pixels_of = pixels_of
        self.inner = inner if inner is not None else runner.SummarySink(digest=False)
        self.samples = {}  # pos -> (cx, cy, n_obs, {pixel: (rows, mask words)})
        self._lock = threading.Lock()

    @property
    def chips(self):
        return self.inner.chips

    def __call__(self, pos, cx, cy, dates, row_offsets, rows, mask_bits):
        keep = {}
        for px in self.pixels_of(pos):
            a, b = int(row_offsets[px]), int(row_offsets[px + 1])
            keep[int(px)] = (rows[a:b].copy(), np.array(mask_bits[px]))
        with self._lock:
            self.samples[int(pos)] = (int(cx), int(cy), int(dates.shape[0]), keep)
        self.inner(pos, cx, cy, dates, row_offsets, rows, mask_bits)


def stratified(pos, n, n_pix=10000, width=100):
    """``n`` pixels of the chip at ``pos`` spread over its rows (n <= the chip's rows: one pixel in
    each of n evenly spaced rows, columns varying with the position and the row)."""
    rows = n_pix // width
    n = min(n, n_pix)
    out = []
    for k in range(n):
        r = (k * rows) // n if n <= rows else k % rows
        c = (int(pos) * 37 + k * 13 + (k // rows) * 29) % width
        out.append(r * width + c)
    return sorted(set(out))


def _compare(dev_rows, dev_mask, u, j, cx, cy, px, words, width=100):
    """one pixel: device rows / mask words vs oracle result u (pixel j of it) -> (int mismatch
    description or None, max relative float difference)"""
    from rows_util import mask_words
    a, b = int(u.seg_offsets[j]), int(u.seg_offsets[j + 1])
    segs = u.segments[a:b]
    exp_n = max(1, b - a)
    if dev_rows.shape[0] != exp_n:
        return 'rows %d vs %d' % (dev_rows.shape[0], exp_n), 0.0
    x, y = cx + 30 * (px % width), cy - 30 * (px // width)
    if not (dev_rows['px'] == x).all() or not (dev_rows['py'] == y).all():
        return 'coordinates', 0.0
    if b == a:
        r = dev_rows[0]
        if not (r['has_model'] == 0 and r['sday'] == 1 and r['eday'] == 1 and r['bday'] == 1):
            return 'default row', 0.0
    else:
        for k, s in enumerate(segs):
            r = dev_rows[k]
            ints = (int(r['sday']), int(r['eday']), int(r['bday']), int(r['curqa']), int(r['has_model']))
            if ints != (int(s['start_day']), int(s['end_day']), int(s['break_day']), int(s['curve_qa']), 1):
                return 'segment %d ints %s vs %s' % (k, ints, (s['start_day'], s['end_day'], s['break_day'],
                                                            s['curve_qa'], 1)), 0.0
    mx = 0.0
    for k, s in enumerate(segs):
        r = dev_rows[k]
        for f, v in (('chprob', s['change_probability']), ('mag', s['magnitude']), ('rmse', s['rmse']),
                     ('intercept', s['intercept']), ('coef', s['coef'])):
            e = np.asarray(v, dtype=np.float64).astype(np.float32).astype(np.float64)
            d = np.asarray(r[f], dtype=np.float64)
            if not np.allclose(d, e, rtol=1e-6, atol=1e-6):
                return 'float: segment %d %s' % (k, f), 0.0
            den = np.maximum(np.abs(e), 1e-6)
            mx = max(mx, float(np.max(np.abs(d - e) / den)) if d.size else 0.0)
    want = mask_words(u.mask[j:j + 1].astype(bool), words)[0]
    if not np.array_equal(np.asarray(dev_mask, dtype='<u4')[:words], want):
        return 'processing mask', mx
    return None, mx


def check(sink, pixel_inputs, threads=16, params=None):
    """Re-detect every sampled pixel with the C oracle and compare.  ``pixel_inputs(pos, pixels)``
    -> (dates [n], spectra [7][k][n] int16, qa [k][n] uint16) of those pixels of the chip at
    ``pos``.  Returns {'pixels', 'chips', 'int_mismatches' (row counts, days, curve QA, coordinates,
    masks), 'float_mismatches' (past 1e-6 relative), 'max_rel', 'first_mismatches'}."""
    from concurrent.futures import ThreadPoolExecutor
    import oracle_ctypes

    def one(pos):
        cx, cy, n_obs, keep = sink.samples[pos]
        pix = sorted(keep)
        d, s, q = pixel_inputs(pos, pix)
        rc, u = oracle_ctypes.detect_batch(d, s, q, params=params, threads=1)
        words = (n_obs + 31) // 32
        bad, mx = [], 0.0
        for j, px in enumerate(pix):
            rows, mask = keep[px]
            why, m = _compare(rows, mask, u, j, cx, cy, px, words)
            mx = max(mx, m)
            if why is not None:
                bad.append((pos, px, why))
        return len(pix), bad, mx

    positions = sorted(sink.samples)
    n, bad, mx = 0, [], 0.0
    with ThreadPoolExecutor(max(1, int(threads))) as ex:
        for k, b, m in ex.map(one, positions):
            n += k
            bad += b
            mx = max(mx, m)
    n_int = sum(1 for b in bad if not b[2].startswith('float:'))
    return {'pixels': n, 'chips': len(positions), 'int_mismatches': n_int, 'float_mismatches': len(bad) - n_int,
            'max_rel': mx, 'first_mismatches': [list(x) for x in bad[:5]]}
