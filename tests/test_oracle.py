"""CPU tests of the oracles themselves (no GPU): the C restatement (oracle/libccdoracle.so)
against the golden vectors minted by the numpy restatement, and the numpy restatement's Lasso
sub-kernel against the installed scikit-learn."""
import warnings

import numpy as np
import pytest

import ccd_ref
import golden_util
import oracle_ctypes
import parity_util
from ccdgpu import abi, synth


@pytest.mark.parametrize('name', golden_util.names())
def test_c_oracle_matches_golden(name):
    (d, s, q), params, ref = golden_util.load(name)
    rc, got = oracle_ctypes.detect_batch(d, s, q, params=params, threads=4)
    assert rc == 0
    problems, max_rel = parity_util.compare(got, ref)
    assert not problems, problems
    assert max_rel < 1e-6


def test_numpy_restatement_reproduces_golden_edges():
    for name in ('ref_fill4', 'ref_ard12', 'mixed_edge'):
        (d, s, q), params, ref = golden_util.load(name)
        for px in range(q.shape[0]):
            r = ccd_ref.detect(d, *[s[b, px] for b in range(7)], q[px], params=params)
            assert abi.PROCEDURES.index(r['procedure']) == ref.procedure[px]
            assert np.array_equal(np.array(r['processing_mask'], dtype=bool), ref.mask[px])
            a, b = ref.seg_offsets[px], ref.seg_offsets[px + 1]
            assert len(r['change_models']) == b - a


def test_lasso_port_matches_installed_sklearn():
    """models/lasso.fitted_model = sklearn Lasso(max_iter=1000).fit on coefficient_matrix:
    the restatement's port of sklearn 0.18's coordinate descent agrees with sklearn 1.7.2."""
    from sklearn.linear_model import Lasso
    P = ccd_ref.get_params()
    d, s, q = synth.chip(synth.config(2), 2, 0, 4)
    o = np.argsort(d)
    d = d[o]
    rng = np.random.default_rng(0)
    worst = 0.0
    for trial in range(60):
        n = int(rng.integers(12, 300))
        st = int(rng.integers(0, len(d) - n))
        k = (4, 6, 8)[trial % 3]
        dd = d[st:st + n]
        y = s[int(rng.integers(0, 7)), int(rng.integers(0, 4))][o][st:st + n].astype(float)
        f = ccd_ref.fitted_model(dd, y, P, k)
        X = ccd_ref.coefficient_matrix(dd, P.AVG_DAYS_YR, k)
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')
            m = Lasso(max_iter=1000).fit(X, y)
        nz = np.abs(m.coef_) > 0
        rel = np.max(np.abs(m.coef_ - f.coef)[nz] / np.abs(m.coef_)[nz]) if nz.any() else 0.0
        worst = max(worst, rel, abs(m.intercept_ - f.intercept) / abs(m.intercept_))
    assert worst < 1e-6, worst


def test_chi2_thresholds():
    """CHANGE/OUTLIER thresholds are chi2.ppf(0.99 / 0.999999, 5); the C oracle's inverse cdf
    (used for the ncompare adjusted threshold) agrees with scipy."""
    from scipy.stats import chi2
    P = ccd_ref.get_params()
    assert P.CHANGE_THRESHOLD == pytest.approx(chi2.ppf(0.99, 5), rel=1e-15)
    assert P.OUTLIER_THRESHOLD == pytest.approx(chi2.ppf(0.999999, 5), rel=1e-15)
    L = oracle_ctypes.lib()
    for peek in (7, 8, 12, 20, 64):
        pt = 1 - (1 - 0.99) ** (6 / peek)
        assert L.ccdoracle_chi2_5_ppf(pt) == pytest.approx(chi2.ppf(pt, 5), rel=1e-12)


def test_oracle_unsupported_qa_is_an_error():
    d, s, q = synth.chip(synth.config(2), 1, 0, 3)
    q = q.copy()
    q[1, 17] = 64  # only bit 6 set: pyccd qa.qabitval raises ValueError
    rc, u = oracle_ctypes.detect_batch(d, s, q, threads=2)
    assert rc == abi.E_QA and u.error_pixel == 1


def test_oracle_peek_overflow_is_an_error():
    """An adaptive peek past CCDGPU_MAX_PEEK (96; only reachable with PEEK_SIZE > 6 on dense
    dates) is CCDGPU_EOVERFLOW, as on the GPU; the default PEEK_SIZE on daily dates (peek 96)
    is supported and matches the golden (test_c_oracle_matches_golden[dense_daily])."""
    (d, s, q), _, _ = golden_util.load('dense_daily')
    rc, _ = oracle_ctypes.detect_batch(d, s[:, :2], q[:2], params={'PEEK_SIZE': 8}, threads=2)
    assert rc == abi.E_OVERFLOW
    assert abi.MAX_PEEK == 96


# ---- the reference's argsort tie order (numpy < 1.17 quicksort)
def _np126_vectors():
    import os
    z = np.load(os.path.join(golden_util.GOLDEN_DIR, 'argsort', 'np126_vectors.npz'))
    off = np.concatenate([[0], np.cumsum(z['lens'])])
    return [(z['keys'][a:b], z['argsort'][a:b]) for a, b in zip(off[:-1], off[1:])]


def test_argsort_restatements_match_real_numpy_quicksort():
    """ccdoracle_np_argsort (C) and ccd_ref.np1_argsort (literal Python port) reproduce the tie
    order of a real numpy's C quicksort (numpy 1.26.4, AVX-512 dispatch off: the aquicksort of
    numpy < 1.25 -- vectors made by tests/golden/argsort/check_np126.py) on closest-DOY keys and
    dates with duplicates, whole and as the first 24 positions of the partial sort."""
    lib = ccd_ref._np1_lib()
    assert lib, 'oracle/libccdoracle.so not built'
    cases = _np126_vectors()
    assert len(cases) >= 100
    for v, ref in cases:
        n = v.shape[0]
        o, deep = ccd_ref.np1_argsort(v)
        assert deep == 0
        assert np.array_equal(o, ref)
        c = np.arange(n, dtype=np.int32)
        lib.ccdoracle_np_argsort(np.ascontiguousarray(v).ctypes.data, c.ctypes.data, n, 0, None)
        assert np.array_equal(c, ref)
        if n > 24:
            c = np.arange(n, dtype=np.int32)
            lib.ccdoracle_np_argsort(np.ascontiguousarray(v).ctypes.data, c.ctypes.data, n, 24, None)
            assert np.array_equal(c[:24], ref[:24])
            assert np.array_equal(ccd_ref.np1_argsort(v, 24)[0][:24], ref[:24])


def test_argsort_stable_option_and_differs_on_ties():
    p = ccd_ref.get_params({'ARGSORT': 'stable'})
    q = ccd_ref.get_params()
    assert q.ARGSORT == 'quicksort'
    v = np.array([3., 1., 2., 1., 3., 1.] * 5)
    assert np.array_equal(ccd_ref.argsort(v, p), np.argsort(v, kind='stable'))
    o = ccd_ref.argsort(v, q)
    assert np.array_equal(v[o], np.sort(v))
    assert not np.array_equal(o, np.argsort(v, kind='stable'))  # quicksort breaks these ties otherwise


def test_pairwise_sum_is_numpys():
    """the C oracle's comparison-rmse sum is numpy's pairwise add.reduce, bit for bit"""
    import ctypes
    lib = ccd_ref._np1_lib()
    lib.ccdoracle_np_pairwise_sum.restype = ctypes.c_double
    lib.ccdoracle_np_pairwise_sum.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    rng = np.random.default_rng(3)
    for n in list(range(0, 40)) + [127, 128, 129, 300, 1000]:
        a = rng.standard_normal(n) ** 2 * 10.0 ** rng.integers(-3, 6, n)
        assert lib.ccdoracle_np_pairwise_sum(np.ascontiguousarray(a).ctypes.data, n) == float(np.sum(a))


def _unpacked_bytes(u):
    return [np.ascontiguousarray(getattr(u, k)).tobytes() for k in ('segments', 'seg_offsets', 'mask', 'procedure', 'probs')]


def test_restatements_never_read_band_values_of_fill_cloud_shadow_observations():
    """The runner's default 'unread' transport encoding (ccdgpu.unread_drop_bits) sends no band
    values for observations whose QA has the fill, cloud or shadow bit, on the premise that no
    procedure reads them (qabitval classes them fill / cloud / shadow whatever else is set, and
    the standard, permanent-snow and insufficient-clear filters keep none of those classes).  Both
    restatements give the same results -- every segment field, mask, procedure and probability,
    bit for bit -- when those band values are replaced by random int16 values: on C2-C5 chips
    (standard and insufficient-clear pixels) and the mixed_edge golden's pixels (all three
    procedures) with the C oracle, and on pixels of each procedure with the numpy restatement
    (pyccd's module structure)."""
    import ccdgpu
    drop, _ = ccdgpu.unread_drop_bits(None)
    assert drop
    rng = np.random.default_rng(6)
    procs = set()
    cases = [(synth.chip(synth.config(cfg), chip, 0, npx), None, nref)
             for cfg, chip, npx, nref in ((3, 1, 120, 2), (4, 2, 200, 4), (5, 3, 80, 1), (2, 4, 120, 2))]
    inputs, params, _ = golden_util.load('mixed_edge')
    cases.append((inputs, params, 6))
    for (d, s, q), params, nref in cases:
        gone = (q & drop) != 0
        assert gone.any() and not gone.all()
        s2 = s.copy()
        s2[:, gone] = rng.integers(-32768, 32768, size=(7, int(gone.sum())), dtype=np.int16)
        rc0, u0 = oracle_ctypes.detect_batch(d, s, q, params=params, threads=4)
        rc1, u1 = oracle_ctypes.detect_batch(d, s2, q, params=params, threads=4)
        assert rc0 == 0 and rc1 == 0
        assert _unpacked_bytes(u0) == _unpacked_bytes(u1)
        procs |= set(int(x) for x in np.asarray(u0.procedure))
        # the numpy restatement on the pixels of each procedure the chip has (at most nref each)
        pick = []
        for pr in sorted(set(int(x) for x in np.asarray(u0.procedure))):
            pick += [int(i) for i in np.flatnonzero(np.asarray(u0.procedure) == pr)[:nref]]
        for px in pick:
            with warnings.catch_warnings():
                warnings.simplefilter('ignore')
                r0 = ccd_ref.detect(d, *[s[b, px] for b in range(7)], q[px], params=params)
                r1 = ccd_ref.detect(d, *[s2[b, px] for b in range(7)], q[px], params=params)
            assert r0['procedure'] == r1['procedure']
            assert list(r0['processing_mask']) == list(r1['processing_mask'])
            assert repr(r0['change_models']) == repr(r1['change_models'])
    assert len(procs) == 3, procs
