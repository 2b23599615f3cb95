"""GPU tests of round 2's batch paths and parity holes (all through the C-ABI, checked against the
C oracle or the golden vectors):

* ragged batches -- chips of different pixel / observation counts in one launch
  (ccdgpu_stage_chips), the layout a real tile (base-cadence + sidelap chips) and a Spark
  partition with several date vectors need;
* the batch row fetch (the tile runner's gather) against the per-chip row fetch;
* per-slot parameters of the double-buffered upload path;
* the adaptive peek beyond the 64-row lookforward batch (dense dates) and its explicit overflow
  error;
* the reference's own chip fixture (C1) through the HIP path for all 10^4 pixels;
* the batched Spark partition function against rows formatted from the oracle;
* every compiled register budget of the detection kernel, and a run with poisoned LDS and slot
  scratch, giving byte-identical results.
"""
import os

import numpy as np
import pytest

import ccdgpu
import golden_util
import oracle_ctypes
import parity_util
from ccdgpu import abi, synth

pytestmark = pytest.mark.gpu

ORACLE_THREADS = 16


@pytest.fixture(scope='module')
def ctx():
    c = ccdgpu.Context(0)
    yield c
    c.close()


def assert_parity(got, ref):
    problems, max_rel = parity_util.compare(got, ref)
    assert not problems, problems[:10]
    assert max_rel < parity_util.RTOL


def tile_mix(n_pix=400):
    """Two base-cadence C3 chips, one sidelap C3 chip and a small C5 sidelap chip: three date
    vectors, two pixel counts."""
    cfg3, cfg5 = synth.config(3), synth.config(5)
    chips = [synth.chip(cfg3, 0, 0, n_pix), synth.chip(cfg3, 1, 0, n_pix), synth.chip(cfg3, 2, 0, n_pix),
             synth.chip(cfg5, 3, 0, 97)]
    assert len({c[0].shape[0] for c in chips}) >= 2
    return chips


def test_ragged_batch_matches_single_chip_runs(ctx):
    chips = tile_mix()
    batch = ctx.stage_chips(chips)
    ctx.run()
    st = ctx.stats()
    assert st['pixels'] == sum(c[2].shape[0] for c in chips)
    got = [ctx.fetch(i) for i in range(len(chips))]
    for i, (d, s, q) in enumerate(chips):
        g = got[i]
        assert g.n_pix == q.shape[0] and g.n_obs == d.shape[0]
        one = ctx.detect_batch(d, s, q)
        assert np.array_equal(g.seg_offsets, one.seg_offsets)
        assert g.segments.tobytes() == one.segments.tobytes()
        assert np.array_equal(g.mask, one.mask)
        rc, ref = oracle_ctypes.detect_batch(d, s, q, threads=ORACLE_THREADS)
        assert rc == 0
        assert_parity(g, ref)
    # staged inputs come back in the ChipBatch layout
    ctx.stage_chips(batch)
    sp, qa = ctx.staged_inputs()
    assert np.array_equal(sp, batch.spectra) and np.array_equal(qa, batch.qa)


def test_batch_rows_equal_per_chip_rows(ctx):
    chips = tile_mix(300)
    batch = ctx.stage_chips(chips)
    ctx.run()
    cx = np.array([3000 * i for i in range(len(chips))], np.int32)
    cy = np.array([-3000 * i for i in range(len(chips))], np.int32)
    off, rows, mask = ctx.fetch_batch_rows(cx, cy)
    assert off.shape == (batch.total_pixels + 1,)
    for c in range(len(chips)):
        o1, r1, m1 = ctx.fetch_rows(c, int(cx[c]), int(cy[c]))
        p0, p1 = int(batch.pix_off[c]), int(batch.pix_off[c + 1])
        assert np.array_equal(off[p0:p1 + 1] - off[p0], o1)
        assert rows[off[p0]:off[p1]].tobytes() == r1.tobytes()
        assert np.array_equal(batch.mask_of(mask, c), m1)
    # the same rows into reusable pinned buffers (ccdgpu_fetch_batch_rows_into), twice into the
    # same buffers
    bufs = ccdgpu.RowsBuffers()
    for _ in range(2):
        o2, r2, m2 = ctx.fetch_batch_rows_into(cx, cy, bufs)
        assert np.array_equal(o2, off) and r2.tobytes() == rows.tobytes() and np.array_equal(m2, mask)


def test_split_run_equals_run_slot(ctx):
    """ccdgpu_run_slot_begin / _query / _end give what ccdgpu_run_slot gives, with another slot
    staged while the detection runs; a second begin before the end is refused."""
    chips = tile_mix(200)
    b = ccdgpu.ChipBatch.from_chips(chips, pinned=True)
    ctx.stage_slot_chips(0, b)
    ctx.run_slot(0)
    ref = [ctx.fetch(i) for i in range(len(chips))]
    ctx.stage_slot_chips(0, b)
    ctx.run_slot_begin(0)
    ctx.stage_slot_chips(1, b)
    with pytest.raises(ccdgpu.CcdGpuError):
        ctx.run_slot_begin(1)
    while not ctx.run_done():
        pass
    ctx.run_slot_end()
    for i in range(len(chips)):
        g = ctx.fetch(i)
        assert g.segments.tobytes() == ref[i].segments.tobytes() and np.array_equal(g.mask, ref[i].mask)
    ctx.run_slot(1)
    assert ctx.fetch(0).segments.tobytes() == ref[0].segments.tobytes()


def test_slots_keep_their_own_params(ctx):
    """staging slot 1 with other params must not change slot 0's pending batch."""
    d, s, q = synth.chip(synth.config(5), 4, 0, 256)
    pa, pb = {'ADAPTIVE_PEEK': False}, {'ADAPTIVE_PEEK': True}
    b = ccdgpu.ChipBatch.from_chips([(d, s, q)], pinned=True)
    ctx.stage_slot_chips(0, b, pa)
    ctx.stage_slot_chips(1, b, pb)
    for slot, p in ((0, pa), (1, pb)):
        ctx.run_slot(slot)
        got = ctx.fetch(0)
        rc, ref = oracle_ctypes.detect_batch(d, s, q, params=p, threads=ORACLE_THREADS)
        assert rc == 0
        assert_parity(got, ref)
    rc, ra = oracle_ctypes.detect_batch(d, s, q, params=pa, threads=ORACLE_THREADS)
    rc, rb = oracle_ctypes.detect_batch(d, s, q, params=pb, threads=ORACLE_THREADS)
    assert ra.segments.tobytes() != rb.segments.tobytes()  # the two settings really differ here


def test_dense_dates_peek_beyond_batch(ctx):
    """Median filtered gap of 1 day: peek 96 (> the 64-row lookforward batch) against the
    numpy restatement's golden and the C oracle; pixel 3 (every other day) peek 48."""
    (d, s, q), params, ref = golden_util.load('dense_daily')
    got = ctx.detect_batch(d, s, q, params=params)
    assert_parity(got, ref)
    rc, oref = oracle_ctypes.detect_batch(d, s, q, params=params, threads=ORACLE_THREADS)
    assert rc == 0
    assert_parity(got, oref)


def test_peek_overflow_is_an_explicit_error(ctx):
    """PEEK_SIZE 8 on daily dates asks for a peek of 128 > CCDGPU_MAX_PEEK: the GPU and the C
    oracle both refuse with CCDGPU_EOVERFLOW instead of silently clamping."""
    (d, s, q), _, _ = golden_util.load('dense_daily')
    with pytest.raises(ccdgpu.CcdGpuError) as ei:
        ctx.detect_batch(d, s, q, params={'PEEK_SIZE': 8})
    assert ei.value.code == abi.E_OVERFLOW
    rc, _ = oracle_ctypes.detect_batch(d, s, q, params={'PEEK_SIZE': 8}, threads=4)
    assert rc == abi.E_OVERFLOW


def test_reference_chip_c1_through_hip_path():
    """C1: the reference's own chip (test/data/chip_response.json: LE07 SRB1 of (-1815585,
    1064805) on 2002-12-21, all fill), its missing layers staged as fill, through the device chip
    packer and detection for all 10^4 pixels.  Every pixel gets the reference test_detect known
    answer (test/test_pyccd.py:129-132): one pyccd.default row, keys == ccd_format_keys,
    cx == -1815585."""
    import json
    from ccdc import pyccd
    from test_reference_boundary import CCD_FORMAT_KEYS
    with open(os.path.join(golden_util.GOLDEN_DIR, 'chipmunk', 'chip_response.json')) as f:
        chips = json.load(f)
    rows = pyccd.detect_chips(chips, symmetric=False)
    assert len(rows) == 10000
    keys = set()
    for i, r in enumerate(rows):
        assert set(r.keys()) == set(CCD_FORMAT_KEYS)
        assert r['cx'] == -1815585 and r['cy'] == 1064805
        assert (r['px'], r['py']) == (-1815585 + 30 * (i % 100), 1064805 - 30 * (i // 100))
        assert r['sday'] == r['eday'] == r['bday'] == '0001-01-01'
        assert r['dates'] == ['2002-12-21'] and r['mask'] == [0]
        assert r['chprob'] is None and r['curqa'] is None and r['blcoef'] is None and r['thint'] is None
        keys.add((r['px'], r['py']))
    assert len(keys) == 10000


def _rows_close(a, b):
    assert a.keys() == b.keys()
    for k in a:
        x, y = a[k], b[k]
        if isinstance(x, float) or isinstance(y, float):
            assert x == pytest.approx(y, rel=parity_util.RTOL, abs=parity_util.ATOL, nan_ok=True), k
        elif isinstance(x, (list, tuple)) and x and isinstance(x[0], float):
            assert list(x) == pytest.approx(list(y), rel=parity_util.RTOL, abs=parity_util.ATOL), k
        else:
            assert x == y, k


def test_detect_partition_against_oracle_rows():
    """f2 (reference pyccd.py:171-183): the batched partition function over records with three
    date vectors in shuffled order -> rows equal to pyccd.format of the C oracle's results."""
    import ccd
    from ccdc import pyccd, timeseries
    chips = tile_mix(60)
    recs, where = [], []
    for c, (d, s, q) in enumerate(chips):
        recs += timeseries.unpack(timeseries.chip_keys(3000 * c, 0, q.shape[0]), d, s, q)
        where += [(c, px) for px in range(q.shape[0])]
    perm = np.random.default_rng(3).permutation(len(recs))
    rows = pyccd.detect_partition([recs[i] for i in perm])
    oracle_by_chip = []
    for d, s, q in chips:
        rc, u = oracle_ctypes.detect_batch(d, s, q, threads=ORACLE_THREADS)
        assert rc == 0
        oracle_by_chip.append(u)
    expected = []
    for i in perm:
        (key, rec), (c, px) = recs[i], where[i]
        expected += pyccd.format(*key, dates=rec['dates'],
                                 ccdresult=abi.pixel_result(oracle_by_chip[c], px, ccd.algorithm))
    assert len(rows) == len(expected) > len(recs)
    for a, b in zip(rows, expected):
        _rows_close(a, b)


def _run_with_env(env, fn):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        c = ccdgpu.Context(0)
        try:
            return fn(c)
        finally:
            c.close()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_kernel_variants_and_poisoned_scratch_are_identical():
    """Every compiled register budget (w1..w4 waves per SIMD) and a run whose LDS block and slot
    scratch are filled with NaN bytes before every pixel give byte-identical results on every
    golden vector (and those results meet the golden parity bar).  Register allocation and stale
    memory cannot leak into a result."""
    names = golden_util.names()
    cases = [golden_util.load(n) for n in names]

    def run_all(c):
        out = []
        for (d, s, q), params, _ in cases:
            u = c.detect_batch(d, s, q, params=params)
            out.append((u.seg_offsets.tobytes(), u.segments.tobytes(), u.mask.tobytes(), u.procedure.tobytes()))
        return out

    base = _run_with_env({'CCDGPU_KERNEL': 'w3', 'CCDGPU_POISON': '0'}, run_all)
    for env in ({'CCDGPU_KERNEL': 'w1'}, {'CCDGPU_KERNEL': 'w2'}, {'CCDGPU_KERNEL': 'w4'},
                {'CCDGPU_KERNEL': 'w3', 'CCDGPU_POISON': '1'}, {'CCDGPU_KERNEL': 'w4', 'CCDGPU_POISON': '1'}):
        env.setdefault('CCDGPU_POISON', '0')
        got = _run_with_env(env, run_all)
        for n, a, b in zip(names, base, got):
            assert a == b, (env, n)
    # and the shared result meets the parity bar against the goldens
    c = ccdgpu.Context(0)
    for (d, s, q), params, ref in cases:
        assert_parity(c.detect_batch(d, s, q, params=params), ref)
    c.close()


_GUARD_SCRIPT = r'''
import hashlib, os, sys
sys.path[:0] = sys.argv[1:]
import ccdgpu, golden_util
from ccdgpu import synth
c = ccdgpu.Context(0)
h = hashlib.sha256()
for name in golden_util.names():
    (d, s, q), params, _ = golden_util.load(name)
    u = c.detect_batch(d, s, q, params=params)
    for a in (u.seg_offsets, u.segments, u.mask, u.procedure):
        h.update(a.tobytes())
for which, chip, n_pix in ((5, 3, 1500), (3, 4, 1500), (4, 11, 1500)):
    d, s, q = synth.chip(synth.config(which), chip, 0, n_pix)
    u = c.detect_batch(d, s, q)
    for a in (u.seg_offsets, u.segments, u.mask, u.procedure):
        h.update(a.tobytes())
c.close()
print(h.hexdigest())
'''


def test_guard_lines_build_trips_no_guard_and_matches_product():
    """The product kernel clamps out-of-range period / scratch indices without recording them;
    the checking build (lib/libccdgpu_guard.so, -DCCD_GUARD_LINES) raises CCDGPU_EHIP naming the
    source line of any tripped guard.  Run in a child process (the library is chosen at load),
    it must trip none on the golden vectors and three synthetic chips (C3 sidelap, C4 high-cloud,
    C5 change-dense), and give byte-identical results to the product build."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    guard = os.path.join(root, 'lcmap-firebird_amd', 'lib', 'libccdgpu_guard.so')
    assert os.path.exists(guard), 'build lib/libccdgpu_guard.so (make -C lcmap-firebird_amd)'
    paths = [os.path.join(root, 'lcmap-firebird_amd'), os.path.join(root, 'tests')]
    outs = []
    for lib in (guard, ccdgpu.LIB_PATH):
        env = dict(os.environ, CCDGPU_LIBRARY=lib)
        r = subprocess.run([sys.executable, '-c', _GUARD_SCRIPT] + paths, env=env, capture_output=True,
                           text=True, timeout=300)
        assert r.returncode == 0, (lib, r.stderr[-2000:])
        outs.append(r.stdout.strip().splitlines()[-1])
    assert outs[0] == outs[1]
