"""Parity comparison between two abi.Unpacked results (GPU vs oracle).

Integer / index outputs must match exactly (procedure, processing mask, segment count, start /
end / break days, observation count, curve QA, change probability); floating point outputs
(coefficients, intercepts, RMSE, magnitudes) within the north-star tolerance: 1e-6 relative
(plus a 1e-9 absolute floor for values that are exactly zero in one result, e.g. Lasso-shrunk
coefficients)."""
import numpy as np

RTOL = 1e-6
ATOL = 1e-9
INT_FIELDS = ('start_day', 'end_day', 'break_day', 'observation_count', 'curve_qa')
FLOAT_FIELDS = ('change_probability', 'magnitude', 'rmse', 'intercept', 'coef')


def compare(got, ref, rtol=RTOL, atol=ATOL, max_report=10):
    """Returns (problems: list[str], max_rel: float)."""
    problems = []
    max_rel = 0.0
    if got.n_pix != ref.n_pix or got.n_obs != ref.n_obs:
        return ['shape %s vs %s' % ((got.n_pix, got.n_obs), (ref.n_pix, ref.n_obs))], np.inf
    if not np.array_equal(got.sorted_dates, ref.sorted_dates):
        problems.append('sorted dates differ')
    if not np.array_equal(got.sort_index, ref.sort_index):
        problems.append('sort index differs')
    for px in range(got.n_pix):
        if len(problems) >= max_report:
            break
        if got.procedure[px] != ref.procedure[px]:
            problems.append('px %d procedure %d vs %d' % (px, got.procedure[px], ref.procedure[px]))
            continue
        if not np.array_equal(got.mask[px], ref.mask[px]):
            d = np.nonzero(got.mask[px] != ref.mask[px])[0]
            problems.append('px %d mask differs at %s (sum %d vs %d)' % (px, d[:8], got.mask[px].sum(), ref.mask[px].sum()))
        ga, gb = got.seg_offsets[px], got.seg_offsets[px + 1]
        ra, rb = ref.seg_offsets[px], ref.seg_offsets[px + 1]
        if gb - ga != rb - ra:
            problems.append('px %d segments %d vs %d: %s vs %s' % (
                px, gb - ga, rb - ra,
                [(s['start_day'], s['end_day'], s['break_day']) for s in got.segments[ga:gb]],
                [(s['start_day'], s['end_day'], s['break_day']) for s in ref.segments[ra:rb]]))
            continue
        for k in range(gb - ga):
            g, r = got.segments[ga + k], ref.segments[ra + k]
            for f in INT_FIELDS:
                if g[f] != r[f]:
                    problems.append('px %d seg %d %s %s vs %s' % (px, k, f, g[f], r[f]))
            for f in FLOAT_FIELDS:
                a, b = np.asarray(g[f], dtype=np.float64), np.asarray(r[f], dtype=np.float64)
                diff = np.abs(a - b)
                scale = np.maximum(np.abs(a), np.abs(b))
                bad = diff > rtol * scale + atol
                with np.errstate(divide='ignore', invalid='ignore'):
                    rel = np.where(scale > 0, diff / scale, 0.0)
                max_rel = max(max_rel, float(np.max(rel)) if rel.size else 0.0)
                if np.any(bad):
                    problems.append('px %d seg %d %s max rel %.3e' % (px, k, f, float(np.max(rel))))
    return problems, max_rel
