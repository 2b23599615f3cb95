"""ctypes mirror of include/ccdgpu.h (structs only) and result unpacking helpers.

The struct layouts here ARE the C-ABI contract of libccdgpu.so; keep them in lock-step with
include/ccdgpu.h.  ``result_to_pixels`` turns a CSR ``ccdgpu_result`` into the per-pixel
``ccd.detect`` result dicts pyccd returns (consumed by ccdc/pyccd.py:106-148 ``format``).
"""
import ctypes

import numpy as np

NBANDS = 7
MAX_OBS = 4096
MAX_PEEK = 96
BANDS = ('blue', 'green', 'red', 'nir', 'swir1', 'swir2', 'thermal')
PROCEDURES = ('standard_procedure', 'permanent_snow_procedure', 'insufficient_clear_procedure')

E_OK, E_INVAL, E_HIP, E_QA, E_NOMEM, E_OVERFLOW = 0, -1, -2, -3, -4, -5

_i32, _u32, _f64 = ctypes.c_int32, ctypes.c_uint32, ctypes.c_double


class Params(ctypes.Structure):
    _fields_ = [
        ('meow_size', _i32), ('peek_size', _i32), ('day_delta', _i32),
        ('coef_min', _i32), ('coef_mid', _i32), ('coef_max', _i32), ('num_obs_factor', _i32),
        ('detection_bands', _u32), ('tmask_bands', _u32), ('lasso_max_iter', _i32),
        ('thermal_min', _i32), ('thermal_max', _i32), ('median_green_filter', _i32),
        ('curve_qa_start', _i32), ('curve_qa_end', _i32), ('curve_qa_insuf_clear', _i32),
        ('curve_qa_persist_snow', _i32),
        ('qa_fill', _i32), ('qa_clear', _i32), ('qa_water', _i32), ('qa_shadow', _i32),
        ('qa_snow', _i32), ('qa_cloud', _i32), ('qa_cirrus1', _i32), ('qa_cirrus2', _i32),
        ('qa_occlusion', _i32), ('qa_bitpacked', _i32), ('adaptive_peek', _i32),
        ('rmse_dof', _i32), ('kelvin_to_celsius', _i32),
        ('avg_days_yr', _f64), ('change_probability', _f64), ('change_threshold', _f64),
        ('outlier_threshold', _f64), ('t_const', _f64), ('lasso_alpha', _f64),
        ('lasso_tol', _f64), ('clear_pct_threshold', _f64), ('snow_pct_threshold', _f64),
        ('argsort_stable', _i32), ('reserved0', _i32),
    ]


class Segment(ctypes.Structure):
    _fields_ = [
        ('start_day', _i32), ('end_day', _i32), ('break_day', _i32),
        ('observation_count', _i32), ('curve_qa', _i32), ('pixel', _i32),
        ('change_probability', _f64),
        ('magnitude', _f64 * NBANDS), ('rmse', _f64 * NBANDS), ('intercept', _f64 * NBANDS),
        ('coef', (_f64 * 7) * NBANDS),
    ]


SEGMENT_DTYPE = np.dtype([
    ('start_day', '<i4'), ('end_day', '<i4'), ('break_day', '<i4'),
    ('observation_count', '<i4'), ('curve_qa', '<i4'), ('pixel', '<i4'),
    ('change_probability', '<f8'),
    ('magnitude', '<f8', (NBANDS,)), ('rmse', '<f8', (NBANDS,)), ('intercept', '<f8', (NBANDS,)),
    ('coef', '<f8', (NBANDS, 7)),
])
assert SEGMENT_DTYPE.itemsize == ctypes.sizeof(Segment)


class Row(ctypes.Structure):
    _fields_ = [
        ('px', _i32), ('py', _i32), ('sday', _i32), ('eday', _i32), ('bday', _i32),
        ('curqa', _i32), ('has_model', _i32), ('chprob', ctypes.c_float),
        ('mag', ctypes.c_float * NBANDS), ('rmse', ctypes.c_float * NBANDS),
        ('coef', (ctypes.c_float * 7) * NBANDS), ('intercept', ctypes.c_float * NBANDS),
    ]


ROW_DTYPE = np.dtype([
    ('px', '<i4'), ('py', '<i4'), ('sday', '<i4'), ('eday', '<i4'), ('bday', '<i4'),
    ('curqa', '<i4'), ('has_model', '<i4'), ('chprob', '<f4'),
    ('mag', '<f4', (NBANDS,)), ('rmse', '<f4', (NBANDS,)), ('coef', '<f4', (NBANDS, 7)),
    ('intercept', '<f4', (NBANDS,)),
])
assert ROW_DTYPE.itemsize == ctypes.sizeof(Row)


class Rows(ctypes.Structure):
    _fields_ = [
        ('n_pix', _i32), ('n_obs', _i32), ('n_rows', ctypes.c_int64),
        ('row_offsets', ctypes.POINTER(ctypes.c_int64)),
        ('rows', ctypes.POINTER(Row)),
        ('mask', ctypes.POINTER(ctypes.c_int8)),
        ('mask_bits', ctypes.POINTER(_u32)),
        ('mask_words', _i32),
    ]


def unpack_rows(r):
    """ccdgpu_rows -> (row_offsets [n_pix+1], rows ROW_DTYPE [n_rows], mask), copied out of
    library memory; mask is int8 [n_pix][n_obs] for a chip fetch, the bit words uint32
    [n_pix][mask_words] for a batch fetch (ccdgpu_fetch_batch_rows)."""
    n_pix, n_obs, n = r.n_pix, r.n_obs, r.n_rows
    off = np.ctypeslib.as_array(r.row_offsets, shape=(n_pix + 1,)).copy()
    # one numpy copy straight out of library memory (numpy releases the GIL for it: the tile
    # runner's worker threads keep issuing uploads meanwhile); no intermediate bytes object
    rows = (np.ctypeslib.as_array(ctypes.cast(r.rows, ctypes.POINTER(ctypes.c_uint8)),
                                  shape=(n * ROW_DTYPE.itemsize,)).view(ROW_DTYPE).copy()
            if n else np.zeros(0, ROW_DTYPE))
    if bool(r.mask_bits):
        w = r.mask_words
        bits = np.ctypeslib.as_array(r.mask_bits, shape=(max(n_pix * w, 1),))[:n_pix * w].reshape(n_pix, w).copy()
        return off, rows, bits
    mask = np.ctypeslib.as_array(r.mask, shape=(n_pix, n_obs)).copy()
    return off, rows, mask


def unpack_mask_bits(bits, n_obs):
    """[n_pix][mask_words] uint32 mask words -> int8 [n_pix][n_obs] (bit i of word i/32)."""
    b = np.ascontiguousarray(bits, dtype='<u4')
    u8 = np.unpackbits(b.view(np.uint8).reshape(b.shape[0], -1), axis=1, bitorder='little')
    return u8[:, :n_obs].astype(np.int8)


class Result(ctypes.Structure):
    _fields_ = [
        ('n_pix', _i32), ('n_obs', _i32), ('n_seg', ctypes.c_int64),
        ('seg_offsets', ctypes.POINTER(ctypes.c_int64)),
        ('segments', ctypes.POINTER(Segment)),
        ('mask_bits', ctypes.POINTER(_u32)),
        ('mask_words', _i32),
        ('procedure', ctypes.POINTER(_i32)),
        ('probs', ctypes.POINTER(_f64)),
        ('sorted_dates', ctypes.POINTER(ctypes.c_int64)),
        ('sort_index', ctypes.POINTER(_i32)),
        ('error_pixel', _i32),
        ('seconds_kernel', _f64), ('seconds_total', _f64),
    ]


class Stats(ctypes.Structure):
    _fields_ = [('detect_ms', _f64), ('prep_ms', _f64), ('pixels', ctypes.c_int64),
                ('segments', ctypes.c_int64), ('lasso_fits', ctypes.c_int64),
                ('cd_sweeps', ctypes.c_int64), ('flops', ctypes.c_int64), ('bytes', ctypes.c_int64),
                ('detect_ms_device', _f64), ('pool_reruns', ctypes.c_int64), ('pool_cap', ctypes.c_int64),
                ('wave_slots', ctypes.c_int64), ('n_cu', ctypes.c_int64)]


# parameter dict keys (pyccd parameters.yaml names) -> Params fields
_PARAM_MAP = {
    'MEOW_SIZE': 'meow_size', 'PEEK_SIZE': 'peek_size', 'DAY_DELTA': 'day_delta',
    'COEFFICIENT_MIN': 'coef_min', 'COEFFICIENT_MID': 'coef_mid', 'COEFFICIENT_MAX': 'coef_max',
    'NUM_OBS_FACTOR': 'num_obs_factor', 'LASSO_MAX_ITER': 'lasso_max_iter',
    'THERMAL_MIN': 'thermal_min', 'THERMAL_MAX': 'thermal_max',
    'MEDIAN_GREEN_FILTER': 'median_green_filter',
    'QA_FILL': 'qa_fill', 'QA_CLEAR': 'qa_clear', 'QA_WATER': 'qa_water',
    'QA_SHADOW': 'qa_shadow', 'QA_SNOW': 'qa_snow', 'QA_CLOUD': 'qa_cloud',
    'QA_CIRRUS1': 'qa_cirrus1', 'QA_CIRRUS2': 'qa_cirrus2', 'QA_OCCLUSION': 'qa_occlusion',
    'QA_BITPACKED': 'qa_bitpacked', 'ADAPTIVE_PEEK': 'adaptive_peek', 'RMSE_DOF': 'rmse_dof',
    'KELVIN_TO_CELSIUS': 'kelvin_to_celsius', 'AVG_DAYS_YR': 'avg_days_yr',
    'CHANGE_PROBABILITY': 'change_probability', 'CHANGE_THRESHOLD': 'change_threshold',
    'OUTLIER_THRESHOLD': 'outlier_threshold', 'T_CONST': 't_const', 'LASSO_ALPHA': 'lasso_alpha',
    'LASSO_TOL': 'lasso_tol', 'CLEAR_PCT_THRESHOLD': 'clear_pct_threshold',
    'SNOW_PCT_THRESHOLD': 'snow_pct_threshold',
}


def default_params():
    p = Params()
    p.meow_size, p.peek_size, p.day_delta = 12, 6, 365
    p.coef_min, p.coef_mid, p.coef_max, p.num_obs_factor = 4, 6, 8, 3
    p.detection_bands, p.tmask_bands = 0x3E, 0x12
    p.lasso_max_iter = 1000
    p.thermal_min, p.thermal_max, p.median_green_filter = -9320, 7070, 400
    p.curve_qa_start, p.curve_qa_end = 14, 24
    p.curve_qa_insuf_clear, p.curve_qa_persist_snow = 44, 54
    (p.qa_fill, p.qa_clear, p.qa_water, p.qa_shadow, p.qa_snow, p.qa_cloud) = (0, 1, 2, 3, 4, 5)
    p.qa_cirrus1, p.qa_cirrus2, p.qa_occlusion = 8, 9, 10
    p.qa_bitpacked, p.adaptive_peek, p.rmse_dof, p.kelvin_to_celsius = 1, 1, 0, 1
    p.avg_days_yr, p.change_probability = 365.2425, 0.99
    p.change_threshold, p.outlier_threshold = 15.086272469388987, 35.888186879610423
    p.t_const, p.lasso_alpha, p.lasso_tol = 4.42, 1.0, 1e-4
    p.clear_pct_threshold, p.snow_pct_threshold = 0.25, 0.75
    p.argsort_stable = 0  # numpy quicksort tie order (the pinned reference's)
    return p


def params_from_dict(d=None):
    """pyccd-style ``params`` dict (parameters.yaml keys) -> Params."""
    p = default_params()
    if not d:
        return p
    for k, v in d.items():
        if k in _PARAM_MAP:
            setattr(p, _PARAM_MAP[k], type(getattr(p, _PARAM_MAP[k]))(v))
        elif k == 'DETECTION_BANDS':
            p.detection_bands = sum(1 << int(b) for b in v)
        elif k == 'TMASK_BANDS':
            p.tmask_bands = sum(1 << int(b) for b in v)
        elif k == 'CURVE_QA':
            p.curve_qa_start = v.get('START', p.curve_qa_start)
            p.curve_qa_end = v.get('END', p.curve_qa_end)
            p.curve_qa_insuf_clear = v.get('INSUF_CLEAR', p.curve_qa_insuf_clear)
            p.curve_qa_persist_snow = v.get('PERSIST_SNOW', p.curve_qa_persist_snow)
        elif k == 'ARGSORT':
            if v not in ('quicksort', 'stable'):
                raise ValueError("ARGSORT must be 'quicksort' or 'stable', not %r" % (v,))
            p.argsort_stable = 1 if v == 'stable' else 0
        elif k in ('FITTER_FN',):
            pass
        else:
            raise KeyError('unsupported ccd parameter %r' % (k,))
    return p


class Unpacked(object):
    """numpy view of a ccdgpu_result (copied out of library memory)."""

    __slots__ = ('n_pix', 'n_obs', 'seg_offsets', 'segments', 'mask', 'procedure', 'probs',
                 'sorted_dates', 'sort_index', 'error_pixel', 'seconds_kernel', 'seconds_total')


def unpack(res):
    u = Unpacked()
    u.n_pix, u.n_obs = res.n_pix, res.n_obs
    n_pix, n_obs, n_seg = res.n_pix, res.n_obs, res.n_seg
    u.seg_offsets = np.ctypeslib.as_array(res.seg_offsets, shape=(n_pix + 1,)).copy()
    if n_seg > 0:
        buf = (ctypes.c_char * (n_seg * SEGMENT_DTYPE.itemsize)).from_address(
            ctypes.addressof(res.segments.contents))
        u.segments = np.frombuffer(bytes(buf), dtype=SEGMENT_DTYPE).copy()
    else:
        u.segments = np.zeros(0, dtype=SEGMENT_DTYPE)
    words = res.mask_words
    bits = np.ctypeslib.as_array(res.mask_bits, shape=(max(n_pix * words, 1),))[:n_pix * words]
    bits = bits.reshape(n_pix, words).astype('<u4')
    mask = np.unpackbits(bits.view(np.uint8).reshape(n_pix, words * 4), axis=1, bitorder='little')
    u.mask = mask[:, :n_obs].astype(bool)
    u.procedure = np.ctypeslib.as_array(res.procedure, shape=(max(n_pix, 1),))[:n_pix].copy()
    u.probs = np.ctypeslib.as_array(res.probs, shape=(max(n_pix * 3, 1),))[:n_pix * 3].reshape(n_pix, 3).copy()
    u.sorted_dates = np.ctypeslib.as_array(res.sorted_dates, shape=(max(n_obs, 1),))[:n_obs].copy()
    u.sort_index = np.ctypeslib.as_array(res.sort_index, shape=(max(n_obs, 1),))[:n_obs].copy()
    u.error_pixel = res.error_pixel
    u.seconds_kernel, u.seconds_total = res.seconds_kernel, res.seconds_total
    return u


def segment_to_change_model(s):
    """One SEGMENT_DTYPE record -> pyccd change_model dict (ccd/change.py results_to_changemodel)."""
    cm = {'start_day': int(s['start_day']), 'end_day': int(s['end_day']),
          'break_day': int(s['break_day']), 'observation_count': int(s['observation_count']),
          'change_probability': float(s['change_probability']), 'curve_qa': int(s['curve_qa'])}
    for b, name in enumerate(BANDS):
        cm[name] = {'magnitude': float(s['magnitude'][b]), 'rmse': float(s['rmse'][b]),
                    'coefficients': tuple(float(x) for x in s['coef'][b]),
                    'intercept': float(s['intercept'][b])}
    return cm


def pixel_result(u, px, algorithm):
    """ccd.detect-compatible dict for pixel ``px`` of an Unpacked batch."""
    a, b = int(u.seg_offsets[px]), int(u.seg_offsets[px + 1])
    probs = u.probs[px]
    return {'algorithm': algorithm,
            'processing_mask': np.asarray(u.mask[px]).astype(np.int64).tolist(),  # (Python ints)
            'procedure': PROCEDURES[int(u.procedure[px])],
            'change_models': [segment_to_change_model(s) for s in u.segments[a:b]],
            'cloud_prob': float(probs[0]), 'snow_prob': float(probs[1]),
            'water_prob': float(probs[2])}
