"""The tile driver on the GPU (ccdc.runner.changedetection; reference core.changedetection,
ccdc/core.py:78-123): chips of the reference tile grid (test/data/tile_response.json) with
synthetic ARD of both cadences, two contexts per GPU with pinned uploads in the transport
encoding, device row packing, per-chip rows gathered -- checked against rows restated from the C
oracle, and byte-identical however the chips are batched, whether they are uploaded encoded or
raw and whether the contexts reserve CUs for their uploads."""
import json
import os

import numpy as np
import pytest

import oracle_ctypes
from rows_util import rows_from_result

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_PIX = 300
N_CHIPS = 8


def tile():
    with open(os.path.join(ROOT, 'tests', 'golden', 'chipmunk', 'tile_response.json')) as f:
        return json.load(f)


def chip(p):
    from ccdgpu import synth
    return synth.chip(synth.config(5 if p % 3 == 2 else 3), p, 0, N_PIX)


def source(pos):
    import ccdgpu
    return ccdgpu.ChipBatch.from_chips([chip(p) for p in pos], pinned=True)


def run(contexts, batch_chips, encode=True, copy_cus=8):
    from ccdc import runner
    sink = runner.SummarySink(keep_rows=True)
    res = runner.changedetection(tile(), source, device=0, contexts=contexts, batch_chips=batch_chips,
                                 number=N_CHIPS, sink=sink, encode=encode, copy_cus=copy_cus)
    return res, sink


def test_tile_runner_rows_match_oracle_and_batching():
    res, sink = run(2, 3)
    t = tile()
    assert res['xys'] == tuple((int(x), int(y)) for x, y in t['chips'][:N_CHIPS])
    assert {c['n_obs'] for c in res['chips']} == {1421, 2121}
    for p in range(N_CHIPS):
        d, s, q = chip(p)
        rc, u = oracle_ctypes.detect_batch(d, s, q, threads=16)
        assert rc == 0
        cx, cy = (int(v) for v in t['chips'][p])
        ro, rr = rows_from_result(u, cx, cy)
        off, rows, mask = sink.rows[p]
        assert np.array_equal(off, ro), p
        for f in ('px', 'py', 'sday', 'eday', 'bday', 'curqa', 'has_model'):
            assert np.array_equal(rows[f], rr[f]), (p, f)
        for f in ('chprob', 'mag', 'rmse', 'intercept', 'coef'):
            np.testing.assert_allclose(rows[f], rr[f], rtol=1e-6, atol=1e-6, err_msg='%d %s' % (p, f))
        assert np.array_equal(mask, u.mask.astype(np.int8)), p
    res2, _ = run(1, 5)
    assert [c['digest'] for c in res2['chips']] == [c['digest'] for c in res['chips']]
    # the runner's default upload is the transport encoding: raw uploads give the same rows
    res3, _ = run(2, 4, encode=False)
    assert [c['digest'] for c in res3['chips']] == [c['digest'] for c in res['chips']]
    # and so do contexts without CUs reserved for the upload stream (ccdgpu_init_copy_cus)
    res4, _ = run(2, 3, copy_cus=0)
    assert [c['digest'] for c in res4['chips']] == [c['digest'] for c in res['chips']]


# ---- full-size chips through the product defaults ---------------------------------------------
FULL_CHIPS = 24


def _full_cfg_id(p):
    """(config, generator chip id) of tile position p: change-dense C5 chips mixed into C3 tile
    chips, ids spread over the tile so both cadences (1421 / 2121 obs) occur"""
    from ccdgpu import synth
    return synth.config(5 if p % 3 == 2 else 3), 97 * p + 11


class _FullSource(object):
    """full 10^4-pixel chips generated on the GPU (one generator per fetch thread), pinned"""

    def __init__(self):
        import threading
        self._local = threading.local()
        self.gens = []

    def __call__(self, positions):
        import ccdgpu
        from ccdgpu import synth
        g = getattr(self._local, 'g', None)
        if g is None:
            g = self._local.g = synth.DeviceGenerator(0)
            self.gens.append(g)
        chips = []
        for p in positions:
            cfg, cid = _full_cfg_id(p)
            chips.append(g.batch(cfg, [cid], n_pix=10000, pinned=False).chip(0))
        return ccdgpu.ChipBatch.from_chips(chips, pinned=True)


def _full_inputs(pos, pixels):
    from ccdgpu import synth
    cfg, cid = _full_cfg_id(pos)
    parts = [synth.chip(cfg, cid, px, 1) for px in pixels]
    d = parts[0][0]
    return d, np.concatenate([s for _, s, _ in parts], axis=1), np.concatenate([q for _, _, q in parts], axis=0)


def test_full_size_tile_with_product_defaults_matches_oracle_on_stratified_pixels():
    """ccdc.runner.changedetection as the tile leg runs it -- 4 contexts per GPU, 6-chip launches,
    8 CUs reserved per context for uploads, the 'unread' transport encoding, upload depth 2, split
    run with staging during detection -- over 24 distinct full-size (10^4-pixel) chips of both
    cadences with change-dense C5 chips mixed in (reference tile loop core.py:97-108 over
    ccd.detect, pyccd.py:168); 100 stratified pixels per chip (one in every row) re-detected by
    the C oracle: rows, days, curve QA, masks bit-exact, floats within 1e-6."""
    import time
    from ccdc import runner
    import tile_sample
    sink = tile_sample.PixelSampleSink(lambda pos: tile_sample.stratified(pos, 100))
    src = _FullSource()
    t = time.time()
    res = runner.changedetection(tile(), src, device=0, number=FULL_CHIPS, sink=sink, tail_chips=4)
    run_s = time.time() - t
    for g in src.gens:
        g.close()
    assert [c['pos'] for c in res['chips']] == list(range(FULL_CHIPS))
    assert {c['n_obs'] for c in res['chips']} == {1421, 2121}
    assert all(c['n_pix'] == 10000 for c in res['chips'])
    st = res['ranks'][0]
    assert st['batches'] <= 8, st  # (full launches, not the tail's quarter batches throughout)
    out = tile_sample.check(sink, _full_inputs, threads=16)
    print('full-size tile parity: %s, runner %.1f s' % (out, run_s))
    assert out['pixels'] >= 100 * FULL_CHIPS - 5 and out['chips'] == FULL_CHIPS
    assert out['int_mismatches'] == 0 and out['float_mismatches'] == 0, out


def test_batch_chain_rows_equal_the_fetched_rows_and_overflow_falls_back():
    """ccdgpu_run_slot_begin_rows / _end_rows (the rows in the detection's device chain) give the
    rows, offsets and mask words of run_slot + fetch_batch_rows_into, byte for byte; with a rows
    buffer too small for the batch (C5 chips: several segments per pixel) the run completes,
    reports the count and the rows are fetched into the grown buffer."""
    import ccdgpu
    from ccdgpu import synth
    cs = [synth.chip(synth.config(5), 3, 0, 400), synth.chip(synth.config(3), 4, 0, 300),
          synth.chip(synth.config(3), 5, 0, 200)]
    enc = ccdgpu.EncodedBatch.encode(cs, threads=4)
    cx, cy = [-1815585, -1812585, -1809585], [1064805, 1064805, 1061805]
    ctx = ccdgpu.Context(0, copy_cus=8)
    try:
        ctx.stage_slot_chips(0, enc)
        ctx.run_slot(0)
        ref = [np.array(a) for a in ctx.fetch_batch_rows_into(cx, cy, ccdgpu.RowsBuffers())]
        for rpp in (2.0, 0.5):
            bufs = ccdgpu.RowsBuffers(rows_per_pixel=rpp)
            ctx.stage_slot_chips(1, enc)
            ctx.run_slot_begin_rows(1, cx, cy, bufs)
            got = ctx.run_slot_end_rows()
            assert np.array_equal(got[0], ref[0]), rpp
            assert got[1].tobytes() == ref[1].tobytes(), rpp
            assert np.array_equal(got[2], ref[2]), rpp
            if rpp < 1:
                assert bufs.rows_per_pixel > rpp  # learned from the overflow
        # the copy size learned from a batch of ~1 row per pixel (C3 chips), then a batch with
        # more rows per pixel than that: the overflow path, the same rows
        bufs = ccdgpu.RowsBuffers()
        enc3 = ccdgpu.EncodedBatch.encode(cs[1:], threads=4)
        ctx.stage_slot_chips(2, enc3)
        ctx.run_slot_begin_rows(2, cx[1:], cy[1:], bufs)
        ctx.run_slot_end_rows()
        assert bufs.copy_per_pixel is not None and bufs.copy_per_pixel < 2.0
        ctx.stage_slot_chips(0, enc)
        ctx.run_slot_begin_rows(0, cx, cy, bufs)
        got = ctx.run_slot_end_rows()
        assert got[1].tobytes() == ref[1].tobytes()
        assert np.array_equal(got[0], ref[0]) and np.array_equal(got[2], ref[2])
    finally:
        ctx.close()
    assert ref[1].shape[0] > 900  # more rows than 0.5 per pixel


# ---- the batch chain's segment-pool overflow rerun ---------------------------------------------
# (ccdgpu_run_slot_end_rows, ccdgpu_api.cpp: the detection reports a pool overflow, the chain's
# CSR / row kernels write nothing -- ccd_rows.hip -- and the host grows the pool and reruns the
# detection and its chain.  The path faulted the card once (the scatter wrote past the CSR
# buffer); these tests drive it on purpose.)
_C5_FULL = (3, 41, 77)  # generator chip ids of full change-dense chips (12.5 segments per pixel)

_POOL_SCRIPT = r'''
import hashlib, os, sys
sys.path[:0] = sys.argv[1:]
import numpy as np
import ccdgpu
from ccdgpu import synth
cs = [synth.chip(synth.config(5), cid, 0, 10000) for cid in (3, 41, 77)]
enc = ccdgpu.EncodedBatch.encode(cs, threads=4)
cx, cy = [-1815585, -1812585, -1809585], [1064805, 1064805, 1061805]
ctx = ccdgpu.Context(0, copy_cus=8)
bufs = ccdgpu.RowsBuffers()
ctx.stage_slot_chips(0, enc)
ctx.run_slot_begin_rows(0, cx, cy, bufs)
off, rows, mask = ctx.run_slot_end_rows()
st = ctx.stats()
ctx.close()
h = hashlib.sha256()
for a in (off, rows, mask):
    h.update(np.ascontiguousarray(a).tobytes())
print(st['pool_reruns'], st['segments'], h.hexdigest())
'''


def _chain_rows(ctx, enc, cx, cy, bufs):
    ctx.stage_slot_chips(0, enc)
    ctx.run_slot_begin_rows(0, cx, cy, bufs)
    return [np.array(a) for a in ctx.run_slot_end_rows()]


def test_batch_chain_pool_overflow_rerun_matches_oracle_and_plain_run():
    """Three full 10^4-pixel C5 chips (12.5 segments per pixel) through run_slot_begin_rows /
    _end_rows on FRESH contexts: with the initial pool at 1 segment per pixel
    (CCDGPU_POOL_PER_PIXEL=1) and at the product's 8, both more than the pool holds, so the
    detection overflows, the chain writes nothing, the host grows the pool and reruns.  The rows,
    offsets and mask words equal a chain-free run_slot + fetch_batch_rows_into on a context whose
    pool already fits, byte for byte; 60 stratified pixels per chip equal the C oracle (reference
    ccd.detect, ccdc/pyccd.py:168; rows as pyccd.format, pyccd.py:106-148); the checking build
    (lib/libccdgpu_guard.so) trips no guard on the same rerun and gives the same bytes."""
    import subprocess
    import sys
    import ccdgpu
    from ccdgpu import synth
    import tile_sample
    cfg = synth.config(5)
    cs = [synth.chip(cfg, cid, 0, 10000) for cid in _C5_FULL]
    enc = ccdgpu.EncodedBatch.encode(cs, threads=4)
    cx, cy = [-1815585, -1812585, -1809585], [1064805, 1064805, 1061805]
    # reference bytes: a context that has already grown its pool (second run), no chain
    ref_ctx = ccdgpu.Context(0, copy_cus=8)
    try:
        ref_ctx.stage_slot_chips(0, enc)
        ref_ctx.run_slot(0)
        ref_ctx.stage_slot_chips(1, enc)
        ref_ctx.run_slot(1)
        assert ref_ctx.stats()['pool_reruns'] == 0  # the pool fits now
        ref = [np.array(a) for a in ref_ctx.fetch_batch_rows_into(cx, cy, ccdgpu.RowsBuffers())]
        n_seg = ref_ctx.stats()['segments']
    finally:
        ref_ctx.close()
    assert n_seg > 8 * 30000, n_seg  # more than the product's initial pool: every fresh context overflows
    for per_pixel in ('1', None):
        old = os.environ.pop('CCDGPU_POOL_PER_PIXEL', None)
        if per_pixel is not None:
            os.environ['CCDGPU_POOL_PER_PIXEL'] = per_pixel
        try:
            ctx = ccdgpu.Context(0, copy_cus=8)
        finally:
            os.environ.pop('CCDGPU_POOL_PER_PIXEL', None)
            if old is not None:
                os.environ['CCDGPU_POOL_PER_PIXEL'] = old
        try:
            got = _chain_rows(ctx, enc, cx, cy, ccdgpu.RowsBuffers())
            st = ctx.stats()
        finally:
            ctx.close()
        assert st['pool_reruns'] >= 1 and st['pool_cap'] >= n_seg, (per_pixel, st)
        assert st['segments'] == n_seg
        assert np.array_equal(got[0], ref[0]), per_pixel
        assert got[1].tobytes() == ref[1].tobytes(), per_pixel
        assert np.array_equal(got[2], ref[2]), per_pixel
    # oracle parity of the rerun's rows on stratified pixels
    sink = tile_sample.PixelSampleSink(lambda pos: tile_sample.stratified(pos, 60))
    off, rows, mask = got
    words = mask.shape[1]
    for c in range(3):
        p0, p1 = 10000 * c, 10000 * (c + 1)
        r0 = int(off[p0])
        sink(c, cx[c], cy[c], cs[c][0], off[p0:p1 + 1] - r0, rows[r0:int(off[p1])], mask[p0:p1])

    def inputs(pos, pixels):
        parts = [synth.chip(cfg, _C5_FULL[pos], px, 1) for px in pixels]
        return (parts[0][0], np.concatenate([s for _, s, _ in parts], axis=1),
                np.concatenate([q for _, _, q in parts], axis=0))
    out = tile_sample.check(sink, inputs, threads=16)
    assert out['pixels'] == 180 and out['int_mismatches'] == 0 and out['float_mismatches'] == 0, out
    assert words == (cs[0][0].shape[0] + 31) // 32
    # the checking build on the same rerun (a child process: the library is chosen at load)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    guard = os.path.join(root, 'lcmap-firebird_amd', 'lib', 'libccdgpu_guard.so')
    h = __import__('hashlib').sha256()
    for a in got:
        h.update(np.ascontiguousarray(a).tobytes())
    paths = [os.path.join(root, 'lcmap-firebird_amd'), os.path.join(root, 'tests')]
    env = dict(os.environ, CCDGPU_LIBRARY=guard, CCDGPU_POOL_PER_PIXEL='1')
    r = subprocess.run([sys.executable, '-c', _POOL_SCRIPT] + paths, env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    reruns, segs, digest = r.stdout.strip().splitlines()[-1].split()
    assert int(reruns) >= 1 and int(segs) == n_seg and digest == h.hexdigest()


def test_c5_only_tile_through_the_runner_takes_the_pool_rerun_and_matches_oracle():
    """ccdc.runner.changedetection with the product defaults over 8 full change-dense (C5) chips:
    every context's first batch overflows the initial segment pool (12.5 segments per pixel
    against 8) and is rerun inside the batch chain; 50 stratified pixels per chip equal the C
    oracle."""
    from ccdc import runner
    import tile_sample
    import ccdgpu
    from ccdgpu import synth
    cfg = synth.config(5)
    reruns = []

    class Recording(ccdgpu.Context):
        def run_slot_end_rows(self):
            out = super(Recording, self).run_slot_end_rows()
            st = self.stats()
            reruns.append((st['pool_reruns'], st['pool_cap'], st['pixels']))
            return out

    def factory(dev):
        return Recording(dev, copy_cus=8)

    class Src(object):
        def __call__(self, positions):
            return ccdgpu.ChipBatch.from_chips([synth.chip(cfg, 1000 + p, 0, 10000) for p in positions],
                                               pinned=True)
    sink = tile_sample.PixelSampleSink(lambda pos: tile_sample.stratified(pos, 50))
    res = runner.changedetection(tile(), Src(), device=0, number=8, sink=sink, context_factory=factory)
    assert [c['pos'] for c in res['chips']] == list(range(8))
    assert reruns and sum(r for r, _, _ in reruns) >= 1, reruns
    assert all(cap >= 8 * px for _, cap, px in reruns)

    def inputs(pos, pixels):
        parts = [synth.chip(cfg, 1000 + pos, px, 1) for px in pixels]
        return (parts[0][0], np.concatenate([s for _, s, _ in parts], axis=1),
                np.concatenate([q for _, _, q in parts], axis=0))
    out = tile_sample.check(sink, inputs, threads=16)
    assert out['pixels'] == 400 and out['int_mismatches'] == 0 and out['float_mismatches'] == 0, out


def test_unsupported_qa_with_rows_overflow_still_raises():
    """A batch with an unsupported bit-packed QA value AND more rows than the chain's rows buffer
    copies (RowsBuffers(rows_per_pixel=0.5)): run_slot_end_rows returns every row and sets
    qa_error (CCDGPU_EQA outranks the short buffer), and the tile runner raises pyccd's
    ValueError (qa.qabitval) for it."""
    import ccdgpu
    from ccdgpu import synth
    d, s, q = synth.chip(synth.config(5), 3, 0, 400)
    q = q.copy()
    q[7, 20] = 64  # bit 6 alone: no pyccd QA class
    batch = ccdgpu.ChipBatch.from_chips([(d, s, q)])
    ctx = ccdgpu.Context(0, copy_cus=8)
    try:
        bufs = ccdgpu.RowsBuffers(rows_per_pixel=0.5)
        ctx.stage_slot_chips(0, batch)
        ctx.run_slot_begin_rows(0, [0], [0], bufs)
        off, rows, mask = ctx.run_slot_end_rows()
        assert ctx.qa_error
        assert rows.shape[0] == int(off[-1]) and rows.shape[0] > 400 * 0.5 + 64
        assert bufs.rows_per_pixel > 0.5
    finally:
        ctx.close()
