"""``ccd`` -- drop-in for lcmap-pyccd's public API, backed by the MI355X kernels.

The reference binds pyccd in exactly two places (ccdc/pyccd.py):
    ccdc/pyccd.py:30    ccd.algorithm
    ccdc/pyccd.py:168   ccd.detect(**second(timeseries))      (kwargs = the ard record,
                                                           test/__init__.py:37-46)
``detect`` keeps pyccd's signature, argument meaning and error behaviour (AssertionError on
mismatched shapes like pyccd's __check_inputs, ValueError on an unsupported bit-packed QA value
like qa.qabitval) and returns pyccd's result dict.  ``detect_batch`` / ``detect_records`` are
the batched entries the Spark ``mapPartitions`` path uses: a partition's pixels, grouped by date
vector, go to the GPU in one launch.
Every call runs on the GPU through libccdgpu.so; there is no CPU fallback.
"""
import numpy as np

import ccdgpu
from ccdgpu import abi

__version__ = '2018.03.12.dev-ncompare.b2'
__name = 'lcmap-pyccd'
algorithm = ':'.join([__name, __version__, 'ccdgpu-mi355x'])

BAND_KWARGS = ('blues', 'greens', 'reds', 'nirs', 'swir1s', 'swir2s', 'thermals')


def _empty_result(n_obs):
    nan = float('nan')
    return {'algorithm': algorithm, 'processing_mask': [0] * n_obs,
            'procedure': 'insufficient_clear_procedure', 'change_models': [],
            'cloud_prob': nan, 'snow_prob': nan, 'water_prob': nan}


def detect(dates, blues, greens, reds, nirs, swir1s, swir2s, thermals, qas,
           prev_results=None, params=None):
    """pyccd ccd.detect: per-pixel change detection.  Returns
    {algorithm, processing_mask (sorted-date order), procedure, change_models, cloud_prob,
    snow_prob, water_prob}."""
    if prev_results is not None:
        raise NotImplementedError('prev_results (incremental update) is not part of the pinned pyccd API')
    dates = np.asarray(dates)
    qas = np.asarray(qas)
    spectra = np.stack([np.asarray(b) for b in (blues, greens, reds, nirs, swir1s, swir2s, thermals)])
    assert dates.ndim == 1
    assert dates.shape == qas.shape
    assert dates.shape[0] == spectra.shape[1]
    n = dates.shape[0]
    if n == 0:
        return _empty_result(0)
    ctx = ccdgpu.default_context()
    u = ctx.detect_batch(dates, spectra.astype(np.int16).reshape(7, 1, n), qas.reshape(1, n), params)
    return abi.pixel_result(u, 0, algorithm)


def detect_batch(dates, spectra, qas, params=None):
    """Batched detect for pixels sharing one date vector.
    dates [n]; spectra [7][n_pix][n] int16 (band-major, obs-contiguous); qas [n_pix][n].
    Returns a list of pyccd result dicts, one per pixel."""
    dates = np.asarray(dates)
    qas = np.asarray(qas)
    if qas.ndim != 2 or dates.ndim != 1 or qas.shape[1] != dates.shape[0]:
        raise AssertionError('dates [n], qas [n_pix][n] expected')
    n_pix, n = qas.shape
    if n == 0:
        return [_empty_result(0) for _ in range(n_pix)]
    u = ccdgpu.default_context().detect_batch(dates, spectra, qas, params)
    return [abi.pixel_result(u, px, algorithm) for px in range(n_pix)]


def detect_groups(groups, params=None):
    """[(dates [n], spectra [7][n_pix][n], qas [n_pix][n]), ...] -- pixel groups with their own
    date vectors -- -> [[result per pixel] per group], all groups in ONE device launch
    (ccdgpu_stage_chips: groups of their own sizes back to back).  Raises ValueError
    (QAValueError) if any pixel has an unsupported QA value."""
    out = [None] * len(groups)
    live = [i for i, g in enumerate(groups) if np.asarray(g[0]).shape[0] > 0]
    for i, g in enumerate(groups):
        if i not in live:
            out[i] = [_empty_result(0) for _ in range(np.asarray(g[2]).shape[0])]
    if live:
        ctx = ccdgpu.default_context()
        ctx.stage_chips([groups[i] for i in live], params)
        ctx.run()
        for c, i in enumerate(live):
            u = ctx.fetch(c)
            if u.error_pixel >= 0:
                raise ccdgpu.QAValueError('unsupported bit-packed QA value (group %d, pixel %d)' % (i, u.error_pixel))
            out[i] = [abi.pixel_result(u, px, algorithm) for px in range(u.n_pix)]
    return out


def detect_records(records, params=None):
    """[(key, {dates, blues..thermals, qas}), ...] -> [(key, result), ...].  Records are grouped
    by date vector (a chip's pixels, as merlin.create builds them) and every group of the call
    runs in one device launch (detect_groups)."""
    # group by date vector: a record's list is compared with each group's first one (a C-level
    # list comparison) under a cheap (length, first, last) key, so a record's dates are converted
    # to an array only when they open a group (merlin's records carry the dates as a list)
    groups = {}
    order = []
    for idx, (key, rec) in enumerate(records):
        dl = rec['dates']
        if isinstance(dl, np.ndarray):
            k = ('a', np.asarray(dl, dtype=np.int64).tobytes())
        else:
            dl = dl if isinstance(dl, list) else list(dl)
            k = (len(dl), dl[0] if dl else None, dl[-1] if dl else None)
        for g in groups.setdefault(k, []):
            if k[0] == 'a' or g[0] is dl or g[0] == dl:
                g[2].append((idx, key, rec))
                break
        else:
            g = (dl, np.asarray(dl, dtype=np.int64), [(idx, key, rec)])
            groups[k].append(g)
            order.append(g)
    arrays, members_of = [], []
    for _, d, members in order:
        n = d.shape[0]
        spectra = np.empty((7, len(members), n), dtype=np.int16)
        qas = np.empty((len(members), n), dtype=np.uint16)
        for j, (_, _, rec) in enumerate(members):
            for b, kw in enumerate(BAND_KWARGS):
                spectra[b, j] = rec[kw]
            qas[j] = rec['qas']
        arrays.append((d, spectra, qas))
        members_of.append(members)
    out = [None] * len(records)
    for members, results in zip(members_of, detect_groups(arrays, params)):
        for (idx, key, _), res in zip(members, results):
            out[idx] = (key, res)
    return out
