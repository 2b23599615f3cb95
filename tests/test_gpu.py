"""GPU parity tests: the HIP path (through the C-ABI) against the golden vectors and the C
oracle, at golden, chip and maximum sizes, plus size-independent properties.  Integer outputs
(procedure, mask, segment count, days, observation counts, curve QA) must be bit-exact; floats
within 1e-6 relative (tests/parity_util.py)."""
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


@pytest.mark.parametrize('name', golden_util.names())
def test_golden(ctx, name):
    (d, s, q), params, ref = golden_util.load(name)
    got = ctx.detect_batch(d, s, q, params=params)
    assert_parity(got, ref)


@pytest.mark.parametrize('which,chip,n_pix', [(2, 0, 10000), (4, 1, 10000), (5, 3, 4000), (3, 5, 2000)])
def test_chip_vs_oracle(ctx, which, chip, n_pix):
    d, s, q = synth.chip(synth.config(which), chip, 0, n_pix)
    got = ctx.detect_batch(d, s, q)
    rc, ref = oracle_ctypes.detect_batch(d, s, q, threads=ORACLE_THREADS)
    assert rc == 0
    assert_parity(got, ref)
    assert got.segments.shape[0] >= n_pix * (10 if which == 5 else 1) * 0.9


@pytest.mark.parametrize('params', [
    {'ADAPTIVE_PEEK': False},
    {'RMSE_DOF': True},
    {'PEEK_SIZE': 8, 'ADAPTIVE_PEEK': False},
    {'T_CONST': 4.89, 'CHANGE_PROBABILITY': 0.95},
    {'DETECTION_BANDS': [1, 3, 4], 'TMASK_BANDS': [2, 4]},
    {'DETECTION_BANDS': [0, 1, 2, 3, 4, 5, 6]},
    {'KELVIN_TO_CELSIUS': False, 'THERMAL_MIN': 1800, 'THERMAL_MAX': 3400},
    {'COEFFICIENT_MAX': 6, 'LASSO_MAX_ITER': 50},
    # tolerances whose float32 pre-check product would be subnormal: the exact test decides
    {'LASSO_TOL': 1e-10, 'LASSO_MAX_ITER': 200},
    {'LASSO_TOL': 1e-40, 'LASSO_MAX_ITER': 60},
])
def test_param_variants_vs_oracle(ctx, params):
    d, s, q = synth.chip(synth.config(5), 4, 0, 300)
    got = ctx.detect_batch(d, s, q, params=params)
    rc, ref = oracle_ctypes.detect_batch(d, s, q, params=params, threads=ORACLE_THREADS)
    assert rc == 0
    assert_parity(got, ref)


def test_max_observations(ctx):
    """CCDGPU_MAX_OBS dates per pixel (every ~3 days over 1982-2017)."""
    n = abi.MAX_OBS
    d = np.linspace(723868, 736694, n).round().astype(np.int64)
    d = np.unique(d)
    d = np.concatenate([d, d[: n - d.shape[0]] + 1])[:n]
    cfg = synth.config(2)
    _, s, q = synth.chip(cfg, 3, 0, 48, chip_dates=d)
    got = ctx.detect_batch(d, s, q)
    rc, ref = oracle_ctypes.detect_batch(d, s, q, threads=ORACLE_THREADS)
    assert rc == 0
    assert_parity(got, ref)
    with pytest.raises(ccdgpu.CcdGpuError):
        dd = np.arange(n + 1, dtype=np.int64) + 723868
        ctx.detect_batch(dd, np.zeros((7, 1, n + 1), np.int16), np.ones((1, n + 1), np.uint16))


def test_input_order_invariance(ctx):
    """Size-independent property: results do not depend on the order merlin delivers dates in."""
    d, s, q = synth.chip(synth.config(5), 2, 0, 2000)
    a = ctx.detect_batch(d, s, q)
    perm = np.random.default_rng(5).permutation(d.shape[0])
    b = ctx.detect_batch(d[perm], s[:, :, perm], q[:, perm])
    assert np.array_equal(a.mask, b.mask)
    assert np.array_equal(a.seg_offsets, b.seg_offsets)
    assert a.segments.tobytes() == b.segments.tobytes()


def test_pixel_batch_independence(ctx):
    """A pixel's result does not depend on which other pixels share its launch."""
    d, s, q = synth.chip(synth.config(2), 6, 0, 512)
    full = ctx.detect_batch(d, s, q)
    for px in (0, 17, 511):
        one = ctx.detect_batch(d, s[:, px:px + 1], q[px:px + 1])
        a, b = full.seg_offsets[px], full.seg_offsets[px + 1]
        assert one.segments.shape[0] == b - a
        x = full.segments[a:b].copy()
        x['pixel'] = 0
        assert x.tobytes() == one.segments.tobytes()
        assert np.array_equal(one.mask[0], full.mask[px])


def test_staged_multichip_matches_single(ctx):
    cfg = synth.config(2)
    chips = [synth.chip(cfg, c, 0, 700) for c in (0, 1, 2)]
    d = np.stack([c[0] for c in chips])
    s = np.stack([c[1] for c in chips])
    q = np.stack([c[2] for c in chips])
    ctx.stage(d, s, q)
    ctx.run()
    st = ctx.stats()
    assert st['pixels'] == 2100 and st['segments'] > 0
    fetched = [ctx.fetch(i) for i in range(3)]
    for i in range(3):
        got = fetched[i]
        ref = ctx.detect_batch(*chips[i])
        assert got.segments.tobytes() == ref.segments.tobytes()
        assert np.array_equal(got.mask, ref.mask)


def test_unsupported_qa_raises_value_error(ctx):
    d, s, q = synth.chip(synth.config(2), 1, 0, 4)
    q = q.copy()
    q[2, 10] = 64
    with pytest.raises(ValueError) as ei:
        ctx.detect_batch(d, s, q)
    assert ei.value.result.error_pixel == 2


def test_ccd_detect_api_and_reference_known_answer():
    """ccd.detect (pyccd signature) and pyccd.detect(timeseries_element) on the GPU:
    reference test_pyccd.py:129-132."""
    import ccd
    from ccdc import pyccd
    from test_reference_boundary import CCD_FORMAT_KEYS, TIMESERIES_ELEMENT
    rows = pyccd.detect(TIMESERIES_ELEMENT)
    assert len(rows) == 1 and rows[0]['cx'] == -1815585
    assert set(rows[0].keys()) == set(CCD_FORMAT_KEYS)
    assert rows[0]['mask'] == [0, 0, 0, 0] and rows[0]['bday'] == '0001-01-01'
    (d, s, q), params, ref = golden_util.load('c5_chip3_sidelap')
    for px in (0, 3):
        r = ccd.detect(d, *[s[b, px] for b in range(7)], q[px], params=params or None)
        a, b = ref.seg_offsets[px], ref.seg_offsets[px + 1]
        assert [cm['break_day'] for cm in r['change_models']] == list(ref.segments['break_day'][a:b])
        assert np.array_equal(np.array(r['processing_mask'], bool), ref.mask[px])
        assert 'lcmap-pyccd' in r['algorithm']
    empty = ccd.detect([], [], [], [], [], [], [], [], [])
    assert empty['change_models'] == [] and empty['processing_mask'] == []
    with pytest.raises(AssertionError):
        ccd.detect([1, 2], [1], [1], [1], [1], [1], [1], [1], [1, 2])


def test_native_library_is_what_ran(ctx):
    d, s, q = synth.chip(synth.config(2), 0, 0, 2)
    ctx.detect_batch(d, s, q)
    maps = open('/proc/self/maps').read()
    assert 'libccdgpu.so' in maps


def test_upload_slots_match_staged_path(ctx):
    """Double-buffered uploads (ccdgpu_stage_slot / ccdgpu_run_slot, copy stream + pinned host
    memory): each batch's results equal the plain staged path's, with the next batch's upload in
    flight during a detection."""
    import ccdgpu as cg
    batches = []
    for seed in (1, 2, 3):
        d, s, q = synth.chip(synth.config(2), seed, 0, 512)
        pd, ps, pq = cg.pinned_empty(d.shape, d.dtype), cg.pinned_empty(s.shape, s.dtype), cg.pinned_empty(q.shape, q.dtype)
        pd[...], ps[...], pq[...] = d, s, q
        batches.append((pd, ps, pq))
    ref = []
    for d, s, q in batches:
        ctx.stage(d[None], s[None], q[None])
        ctx.run()
        ref.append(ctx.fetch(0))
    ctx.stage_slot(0, batches[0][0][None], batches[0][1][None], batches[0][2][None])
    for i in range(3):
        if i + 1 < 3:
            nd, ns, nq = batches[i + 1]
            ctx.stage_slot((i + 1) & 1, nd[None], ns[None], nq[None])
        ctx.run_slot(i & 1)
        got = ctx.fetch(0)
        assert np.array_equal(got.seg_offsets, ref[i].seg_offsets)
        assert got.segments.tobytes() == ref[i].segments.tobytes()
        assert np.array_equal(got.mask, ref[i].mask)


def test_concurrent_contexts_on_one_device():
    """Two contexts on one device detecting from two host threads at once (own streams, buffers
    and launch-argument slots) give the same results as one context alone."""
    import threading
    batches = [synth.chip(synth.config(c), 7, 0, 1500) for c in (2, 5)]
    ref = []
    solo = ccdgpu.Context(0)
    for d, s, q in batches:
        ref.append(solo.detect_batch(d, s, q))
    solo.close()
    ctxs = [ccdgpu.Context(0), ccdgpu.Context(0)]
    got = [None, None]

    def work(i):
        for _ in range(3):
            got[i] = ctxs[i].detect_batch(*batches[i])

    th = [threading.Thread(target=work, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for c in ctxs:
        c.close()
    for g, r in zip(got, ref):
        assert np.array_equal(g.seg_offsets, r.seg_offsets)
        assert g.segments.tobytes() == r.segments.tobytes()
        assert np.array_equal(g.mask, r.mask)


def test_cu_reservation_extremes_keep_both_stream_masks_nonempty():
    """ccdgpu_init_copy_cus with a reservation near the CU count: every group of CUs keeps at least
    one for the detection and reserves at least one (the reservation is clamped, never empty on
    either side), and the detection is the unreserved one's."""
    d, s, q = synth.chip(synth.config(3), 9, 0, 200)
    ref = ccdgpu.Context(0)
    r = ref.detect_batch(d, s, q)
    ref.close()
    for cus in (1, 255):
        ctx = ccdgpu.Context(0, copy_cus=cus)
        try:
            g = ctx.detect_batch(d, s, q)
        finally:
            ctx.close()
        assert g.segments.tobytes() == r.segments.tobytes(), cus
        assert np.array_equal(g.mask, r.mask), cus


def test_reference_ard_record_through_hip_path():
    """The one multi-date ARD record the reference holds (ccdc/timeseries.py:105-115: merlin's
    layout -- 12 observations, dates descending, -9999 fill, qas 1 / 66 / 322) through
    ccdc.pyccd.detect (pyccd.py:151-168) and ccd.detect on the GPU: the same procedure, processing
    mask (sorted-date order), models and probabilities as the C oracle and the numpy restatement
    (golden ref_ard12); pyccd.format's row carries the input-order ISO dates and the sorted mask."""
    import datetime
    import ccd
    import ccd_ref
    from ccdc import pyccd
    sys_path_golden()
    import make_golden
    rec = dict((k, np.array(v, dtype=np.uint16 if k == 'qas' else np.int16)) for k, v in make_golden.REF_ARD12.items()
               if k != 'dates')
    rec['dates'] = list(make_golden.REF_ARD12['dates'])
    (d, s, q), params, gold = golden_util.load('ref_ard12')
    r = ccd.detect(**rec)
    cpu = ccd_ref.detect(np.array(rec['dates']), *[rec[k] for k in make_golden.BAND_KEYS], rec['qas'])
    rc, orc = oracle_ctypes.detect_batch(d, s, q, threads=1)
    assert rc == 0
    assert r['procedure'] == cpu['procedure'] == abi.PROCEDURES[int(orc.procedure[0])] == 'standard_procedure'
    assert list(map(int, r['processing_mask'])) == list(map(int, cpu['processing_mask'])) == \
        list(orc.mask[0].astype(int)) == list(gold.mask[0].astype(int))
    assert r['change_models'] == cpu['change_models'] == []
    for k in ('cloud_prob', 'snow_prob', 'water_prob'):
        assert r[k] == pytest.approx(cpu[k], rel=1e-12)
    # 4 clear of 12 (fill otherwise): too few for a model window -> pyccd.default's row
    assert sum(r['processing_mask']) == 4
    rows = pyccd.detect(((-1815585, 1064805, -1815585, 1064805), rec))
    assert len(rows) == 1
    row = rows[0]
    assert row['sday'] == row['eday'] == row['bday'] == '0001-01-01'
    assert row['dates'] == [datetime.date.fromordinal(x).isoformat() for x in rec['dates']]
    srt = np.argsort(np.array(rec['dates']), kind='stable')
    assert row['mask'] == [int(rec['qas'][i] in (66, 322)) for i in srt]
    assert list(map(int, row['mask'])) == list(gold.mask[0].astype(int))


def sys_path_golden():
    import os
    import sys
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
    if p not in sys.path:
        sys.path.insert(0, p)
