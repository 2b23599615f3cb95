"""Regenerate the golden vectors in tests/golden/ from oracle/ccd_ref.py (the numpy restatement
of lcmap-pyccd ccd.detect).  Inputs come from the synthetic ARD generator (libccdsynth) plus
hand-built edge cases; expected outputs are the restatement's change models and masks.

    python tests/golden/make_golden.py            # ~1 min on 8 cores
    python tests/golden/make_golden.py dense_daily # one case

The reference itself (lcmap-pyccd) is not importable in this container, so these
vectors pin the GPU path and the C oracle to the restatement; the restatement is pinned by the
reference's own boundary tests (tests/test_reference_boundary.py) and its argsort by a real
numpy's quicksort (tests/golden/argsort/).  Default parameters = ARGSORT 'quicksort' (numpy's
tie order, round 6); the *_stable cases keep the stable rule of rounds 1-5 covered."""
import json
import multiprocessing
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, 'lcmap-firebird_amd'), os.path.join(ROOT, 'oracle')]

import numpy as np  # noqa: E402

import ccd_ref  # noqa: E402
from ccdgpu import abi, synth  # noqa: E402


def run_pixel(args):
    d, spec, q, params = args
    r = ccd_ref.detect(d, *[spec[b] for b in range(7)], q, params=params)
    return r


def to_arrays(results, n_obs):
    P = len(results)
    words = (n_obs + 31) // 32
    procedure = np.array([abi.PROCEDURES.index(r['procedure']) for r in results], dtype=np.int32)
    mask = np.array([r['processing_mask'] for r in results], dtype=np.uint8).reshape(P, n_obs)
    offsets = np.zeros(P + 1, dtype=np.int64)
    segs = []
    for i, r in enumerate(results):
        for cm in r['change_models']:
            s = np.zeros((), dtype=abi.SEGMENT_DTYPE)
            for f in ('start_day', 'end_day', 'break_day', 'observation_count', 'curve_qa'):
                s[f] = cm[f]
            s['pixel'] = i
            s['change_probability'] = cm['change_probability']
            for b, name in enumerate(abi.BANDS):
                s['magnitude'][b] = cm[name]['magnitude']
                s['rmse'][b] = cm[name]['rmse']
                s['intercept'][b] = cm[name]['intercept']
                s['coef'][b] = cm[name]['coefficients']
            segs.append(s)
        offsets[i + 1] = len(segs)
    segments = np.array(segs, dtype=abi.SEGMENT_DTYPE) if segs else np.zeros(0, dtype=abi.SEGMENT_DTYPE)
    probs = np.array([[r['cloud_prob'], r['snow_prob'], r['water_prob']] for r in results], dtype=np.float64)
    return dict(procedure=procedure, mask=np.packbits(mask, axis=1, bitorder='little'),
                seg_offsets=offsets, segments=segments, probs=probs)


def synth_case(which, chip, n_pix, **over):
    cfg = synth.config(which, **over)
    return synth.chip(cfg, chip, 0, n_pix)


REF_ARD12 = {  # values of the docstring example at reference ccdc/timeseries.py:105-115 (data)
    'blues': [-9999, 295, -9999, 204, -9999, 238, -9999, -9999, 195, -9999, -9999, -9999],
    'greens': [-9999, 499, -9999, 422, -9999, 363, -9999, -9999, 334, -9999, -9999, -9999],
    'reds': [-9999, 413, -9999, 324, -9999, 315, -9999, -9999, 264, -9999, -9999, -9999],
    'nirs': [-9999, 2329, -9999, 2379, -9999, 2115, -9999, -9999, 1629, -9999, -9999, -9999],
    'swir1s': [-9999, 1322, -9999, 1205, -9999, 1100, -9999, -9999, 743, -9999, -9999, -9999],
    'swir2s': [-9999, 593, -9999, 593, -9999, 522, -9999, -9999, 375, -9999, -9999, -9999],
    'thermals': [-9999, 3020, -9999, 2930, -9999, 2902, -9999, -9999, 2920, -9999, -9999, -9999],
    'qas': [1, 66, 1, 322, 1, 66, 1, 1, 66, 1, 1, 1],
    'dates': [734992, 734991, 734984, 734983, 734976, 734975, 734448, 734441, 734439, 727265, 726648, 726616],
}
BAND_KEYS = ('blues', 'greens', 'reds', 'nirs', 'swir1s', 'swir2s', 'thermals')


def ref_ard12():
    r = REF_ARD12
    d = np.array(r['dates'], dtype=np.int64)
    s = np.array([r[k] for k in BAND_KEYS], dtype=np.int16)[:, None, :]
    q = np.array(r['qas'], dtype=np.uint16)[None, :]
    return d, s, q


def edge_cases():
    """Hand-built inputs exercising the branches the reference's tests and pyccd's procedures
    name: the reference's all-fill element, few observations, insufficient clear, permanent
    snow, duplicate dates, shuffled dates, L8 cirrus/occlusion QA, int16 thermal wrap."""
    cases = {}
    # reference test/__init__.py:37-46 timeseries_element (4 obs, qa = 1 fill)
    d = np.array([734973, 731205, 724404, 723868], dtype=np.int64)
    cases['ref_fill4'] = (d, np.full((7, 1, 4), -9999, dtype=np.int16), np.ones((1, 4), dtype=np.uint16))
    # reference ccdc/timeseries.py:105-115: the one merlin ARD record the reference holds (12 obs,
    # dates descending as merlin emits them, -9999 fill, qas 1 / 66 / 322); band order blue,
    # green, red, nir, swir1, swir2, thermal
    cases['ref_ard12'] = ref_ard12()
    base_d, base_s, base_q = synth_case(2, 5, 8)
    n = base_d.shape[0]
    order = np.argsort(base_d)
    # few observations: only the last 20 dates clear -> END catch only
    s1, q1 = np.full((7, 1, n), -9999, dtype=np.int16), np.ones((1, n), dtype=np.uint16)
    q1[0, order[-20:]] = 66
    s1[:, 0, order[-20:]] = base_s[:, 1, order[-20:]].clip(100, 5000)
    s1[6, 0, order[-20:]] = 2950
    # insufficient clear: 15 % clear, rest cloud
    rng = np.random.default_rng(7)
    s2, q2 = base_s[:, 2:3].copy(), np.full((1, n), 224, dtype=np.uint16)
    pick = rng.choice(n, size=int(0.15 * n), replace=False)
    q2[0, pick] = 66
    s2[:, 0, pick] = np.array([500, 800, 700, 2800, 2000, 1200, 2900], dtype=np.int16)[:, None] + rng.integers(-40, 40, size=(7, pick.size)).astype(np.int16)
    # permanent snow: 10 % clear, 70 % snow
    s3, q3 = s2.copy(), np.full((1, n), 224, dtype=np.uint16)
    q3[0, pick[:len(pick) * 2 // 3]] = 66
    snow = rng.choice(np.setdiff1d(np.arange(n), pick), size=int(0.7 * n), replace=False)
    q3[0, snow] = 80
    s3[:, 0, snow] = np.array([6000, 6200, 6300, 5500, 400, 300, 2600], dtype=np.int16)[:, None]
    spectra = np.concatenate([s1, s2, s3, base_s[:, 3:6]], axis=1)
    qa = np.concatenate([q1, q2, q3, base_q[3:6]], axis=0)
    # pixel 5: L8 cirrus (768 = bits 8,9) / occlusion (1024) values on its clear obs
    qa[4, order[-60::3]] = 768
    qa[4, order[-59::3]] = 1024
    # pixel 5: hot thermal (K*10 > 3276.7 wraps in int16 after *10-27315)
    spectra[6, 5, order[200:260:5]] = 3400
    cases['mixed_edge'] = (base_d, spectra, qa)
    # duplicate dates: every 10th date duplicated (copy with different values), shuffled input order
    dd = np.concatenate([base_d, base_d[::10]])
    ss = np.concatenate([base_s[:, :4], base_s[:, 4:8, ::10]], axis=2)
    qq = np.concatenate([base_q[:4], base_q[4:8, ::10]], axis=1)
    perm = np.random.default_rng(11).permutation(dd.shape[0])
    cases['dup_shuffled'] = (dd[perm], ss[:, :, perm], qq[:, perm])
    return cases


def dense_case():
    """Daily acquisitions for five years with few clouds: the filtered dates' median gap is 1
    day, so the ncompare peek is round(6 * 16 / 1) = 96 (CCDGPU_MAX_PEEK; larger than the 64-row
    lookforward batch) and the change threshold chi2.ppf(1 - 0.01^(6/96), 5); breaks every 3
    years.  Pixel 3 thins its clear days to every other one (peek 48)."""
    d = np.arange(730120, 730120 + 1826, dtype=np.int64)[::-1].copy()
    cfg = synth.config(5, p_clear=0.93, p_cloud=0.02, p_shadow=0.01, p_snow=0.01, p_water=0.01, p_fill=0.02)
    _, s, q = synth.chip(cfg, 7, 0, 6, chip_dates=d)
    q = q.copy()
    q[3, 1::2] = 224  # every other day cloudy
    return d, s, q


def _tie_years_dates():
    rng = np.random.default_rng(1461)
    days = np.sort(rng.choice(1461, size=46, replace=False))
    return np.concatenate([723900 + 1461 * c + days for c in range(9)]).astype(np.int64)


def _tie_years_pixel(seed, d):
    """one candidate pixel (ascending dates): seasonal cycle + random walk (+ steps every ~3 years
    for odd seeds), optical bands kept inside (0, 10000) by redrawing"""
    rng = np.random.default_rng(seed)
    n = d.shape[0]
    w = 2 * np.pi / 365.2425
    base = np.array([500, 800, 700, 2800, 2000, 1200, 2950], dtype=np.float64)
    amp = np.array([150, 200, 250, 600, 400, 300, 0], dtype=np.float64)
    walk = np.array([25, 30, 35, 60, 50, 40, 0], dtype=np.float64)
    while True:
        y = (base[:, None] + amp[:, None] * np.cos(w * d[None, :] + rng.uniform(0, 2 * np.pi, (7, 1)))
             + np.cumsum(rng.normal(0.0, 1.0, (7, n)), axis=1) * walk[:, None]
             + rng.normal(0.0, 8.0, (7, n)))
        if seed % 2:
            for tb in range(int(d[0]) + 1000, int(d[-1]), 1100):
                y[:, d >= tb] += rng.choice([-1, 1], size=(7, 1)) * rng.uniform(0.1, 0.3, (7, 1)) * base[:, None]
        y[6] = base[6] + rng.normal(0.0, 20.0, n)  # thermal (K x 10) inside the valid range
        if y[:6].min() >= 20 and y[:6].max() <= 9900:
            break
    r = rng.uniform(size=n)
    qa = np.where(r < 0.85, 66, np.where(r < 0.97, 224, 1)).astype(np.uint16)
    y[:, qa == 1] = -9999
    return np.round(y).astype(np.int16), qa


def _tie_years_outcome(args):
    d, sp, qp, params = args
    r = ccd_ref.detect(d, *[sp[b] for b in range(7)], qp, params=params)
    return (tuple(r['processing_mask']),
            tuple((m['start_day'], m['end_day'], m['break_day'], m['observation_count']) for m in r['change_models']))


_TIE_YEARS = None


def tie_years_case():
    """Dates that repeat every 1461 days (4 years: the same 46 days of each 4-year cycle, for 36
    years, descending): find_closest_doy's key |round(d/365.25)*365.25 - d| of two dates 1461
    days apart is equal, so the fit-window entries come in groups of up to nine equal keys and
    the 24 closest almost always cut a group -- numpy's argsort tie order (ARGSORT) decides which
    of its entries enter the comparison rmse (change.lookforward).  The comparison rmse matters
    only where it exceeds the variogram, so the spectra carry a random walk (small consecutive
    differences, large residuals about any harmonic model).  Of 384 candidate pixels the first 8
    whose restated outputs differ between the quicksort and the stable tie rule are kept, and 8
    whose outputs agree."""
    global _TIE_YEARS
    if _TIE_YEARS is None:
        d = _tie_years_dates()
        NC = 384
        cands = [_tie_years_pixel(1000 + k, d) for k in range(NC)]
        jobs = [(d, sp, qp, par) for sp, qp in cands for par in (None, {'ARGSORT': 'stable'})]
        with multiprocessing.Pool(min(8, os.cpu_count() or 1)) as pool:
            outs = pool.map(_tie_years_outcome, jobs)
        diff = [k for k in range(NC) if outs[2 * k] != outs[2 * k + 1]]
        same = [k for k in range(NC) if outs[2 * k] == outs[2 * k + 1]]
        pick = diff[:8] + same[:16 - len(diff[:8])]
        print('tie_years: %d of %d candidates differ between the tie rules; kept %s' % (len(diff), NC, pick))
        s = np.stack([cands[k][0] for k in pick], axis=1)
        q = np.stack([cands[k][1] for k in pick], axis=0)
        _TIE_YEARS = (d[::-1].copy(), s[:, :, ::-1].copy(), q[:, ::-1].copy())
    return _TIE_YEARS


def tie_cycles_case():
    """find_closest_doy with more tied entries than a wave holds: 30 four-year cycles of the same
    40 dates 16 days apart (120 years, 1200 observations, descending).  Every date shares its
    day-of-4-years bin with its copies in the other cycles, so once a fit window spans ~22 of
    them the reference date's own bin holds fewer than 24 entries and the two bins 16 days away
    hold ~22 each: the entries at the cut-off distance number more than 40 and the selection
    more than 64 -- coop_comp's multi-chunk loop, and with ARGSORT='stable' its rank from reloaded
    bucket records.  The kernel needs the exact comparison rmse only for steps its bounds leave
    open, i.e. where the comparison rmse is well above the variogram: the pixels carry a 7-year
    oscillation of amplitude 100 (smooth: a small variogram, residuals about the harmonic model
    well above it) and 5 % clear spikes of 200-600.  Measured with the diagnostic build
    (tools/coop_ties.py): 63 exact comparison rmse steps on these 8 pixels, 56 with more ties
    at the cut-off than needed, 2 selecting more than 64 entries."""
    d = np.concatenate([693600 + 1461 * c + 16 * np.arange(40) for c in range(30)]).astype(np.int64)
    n = d.shape[0]
    w = 2 * np.pi / 365.2425
    base = np.array([500, 800, 700, 2800, 2000, 1200, 2950.])
    amp = np.array([150, 200, 250, 600, 400, 300, 0.])
    S, Q = [], []
    for k in range(8):
        rng = np.random.default_rng(5000 + k)
        y = base[:, None] + amp[:, None] * np.cos(w * d[None, :] + rng.uniform(0, 2 * np.pi, (7, 1))) + rng.normal(0, 8, (7, n))
        y[:6] += 100 * np.sin(2 * np.pi * d[None, :] / (7 * 365.25) + rng.uniform(0, 2 * np.pi, (6, 1)))
        sp = rng.uniform(size=n) < 0.05
        y[:6, sp] += rng.choice([-1, 1], size=(6, sp.sum())) * rng.uniform(200, 600, (6, sp.sum()))
        y[6] = base[6] + rng.normal(0, 20, n)
        y[:6] = np.clip(y[:6], 20, 9900)
        S.append(np.round(y).astype(np.int16))
        Q.append(np.full(n, 66, np.uint16))
    s = np.stack(S, axis=1)
    q = np.stack(Q, axis=0)
    return d[::-1].copy(), s[:, :, ::-1].copy(), q[:, ::-1].copy()


def main():
    only = set(sys.argv[1:])
    cases = {
        'c2_chip11': (synth_case(2, 11, 16), None),
        'c4_chip11': (synth_case(4, 11, 16), None),
        'c5_chip3_sidelap': (synth_case(5, 3, 10), None),
        'c3_chip4_sidelap': (synth_case(3, 4, 6), None),
        'c5_chip11_fixedpeek': (synth_case(5, 11, 8), {'ADAPTIVE_PEEK': False}),
        'c2_chip11_rmsedof': (synth_case(2, 11, 6), {'RMSE_DOF': True}),
    }
    for name, inp in edge_cases().items():
        cases[name] = (inp, None)
    cases['dense_daily'] = (dense_case(), None)
    cases['tie_years'] = (tie_years_case(), None)
    cases['tie_years_stable'] = (tie_years_case(), {'ARGSORT': 'stable'})
    cases['dup_shuffled_stable'] = (cases['dup_shuffled'][0], {'ARGSORT': 'stable'})
    cases['tie_cycles'] = (tie_cycles_case(), None)
    cases['tie_cycles_stable'] = (tie_cycles_case(), {'ARGSORT': 'stable'})
    with multiprocessing.Pool(min(8, os.cpu_count() or 1)) as pool:
        for name, ((d, s, q), params) in cases.items():
            if only and name not in only:
                continue
            jobs = [(d, s[:, p], q[p], params) for p in range(q.shape[0])]
            results = pool.map(run_pixel, jobs)
            out = to_arrays(results, d.shape[0])
            order = ccd_ref.argsort(d, ccd_ref.get_params(params)).astype(np.int32)  # ccd.detect's date sort
            np.savez_compressed(os.path.join(HERE, name + '.npz'), dates=d, spectra=s, qa=q,
                                params=np.array(json.dumps(params or {})), sort_index=order, **out)
            print(name, 'pixels', q.shape[0], 'obs', d.shape[0], 'segments', len(out['segments']),
                  'procedures', np.bincount(out['procedure'], minlength=3).tolist(), flush=True)


if __name__ == '__main__':
    main()
