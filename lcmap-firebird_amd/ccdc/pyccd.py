"""ccdc.pyccd -- the change-detection plugin boundary (mirror of reference ccdc/pyccd.py).

Same names, signatures and row dicts as the reference (pyccd.py:27-183).  The only behavioural
difference is the backend: ``ccd`` here is the MI355X shim (lcmap-firebird_amd/ccd), and ``rdd``
batches each Spark partition's pixels by shared date vector (``mapPartitions``) instead of one
``ccd.detect`` per pixel (``flatMap``, pyccd.py:183); the rows produced are identical.
pyspark, cytoolz and merlin are optional here: the helpers they supplied are restated below.
"""
from datetime import date

import numpy as np

import ccd
from ccdc import logger
from ccdc._types import (ArrayType, ByteType, FloatType, IntegerType, StringType, StructField,
                         StructType, require_pyspark)

_NO_DEFAULT = object()


# ---- cytoolz / merlin.functions helpers used by the reference module -------------------------
def first(seq):
    return next(iter(seq))


def second(seq):
    it = iter(seq)
    next(it)
    return next(it)


def get(key, coll, default=_NO_DEFAULT):
    """cytoolz.get: coll[key], or default when given and the key is missing."""
    try:
        return coll[key]
    except (KeyError, IndexError, TypeError):
        if default is _NO_DEFAULT:
            raise
        return default


def get_in(keys, coll, default=None):
    """cytoolz.get_in."""
    try:
        for k in keys:
            coll = coll[k]
        return coll
    except (KeyError, IndexError, TypeError):
        return default


_NATIVE = frozenset((int, float, str, bool, type(None)))


def denumpify(arg):
    """merlin.functions.denumpify: numpy scalars/arrays -> native Python, containers kept.  A list
    or tuple of native scalars (a row's ISO dates, its mask) is copied in one pass instead of one
    recursive call per element -- the same result."""
    if isinstance(arg, np.generic):
        return arg.item()
    if isinstance(arg, np.ndarray):
        return arg.tolist()
    if isinstance(arg, dict):
        return {k: denumpify(v) for k, v in arg.items()}
    if isinstance(arg, list):
        if _NATIVE.issuperset(map(type, arg)):
            return list(arg)
        return [denumpify(v) for v in arg]
    if isinstance(arg, tuple):
        if _NATIVE.issuperset(map(type, arg)):
            return tuple(arg)
        return tuple(denumpify(v) for v in arg)
    return arg


_iso_memo = {}


def _iso_dates(dates):
    """[date.fromordinal(o).isoformat() for o in dates] as a new list, the strings of a date
    vector built once: a chip's pixels (and a partition's records of one chip) share it, and the
    conversion is most of a row's formatting time otherwise."""
    if not isinstance(dates, (list, tuple, np.ndarray)):
        dates = list(dates)  # (an iterator: one pass for the key, one for the strings)
    key = tuple(dates)
    iso = _iso_memo.get(key)
    if iso is None:
        iso = [date.fromordinal(o).isoformat() for o in dates]
        if len(_iso_memo) >= 16:
            _iso_memo.clear()
        _iso_memo[key] = iso
    return list(iso)


# ---- reference API ------------------------------------------------------------------------------
def algorithm():
    """Returns The ccd algorithm and version (pyccd.py:27-30)."""
    return ccd.algorithm


def table():
    """Cassandra pyccd table name (pyccd.py:33-36)."""
    return 'data'


def schema():
    """Spark schema of the ccd dataframe (pyccd.py:39-81)."""
    return StructType([
        StructField('cx', IntegerType(), nullable=False),
        StructField('cy', IntegerType(), nullable=False),
        StructField('px', IntegerType(), nullable=False),
        StructField('py', IntegerType(), nullable=False),
        StructField('sday', StringType(), nullable=False),
        StructField('eday', StringType(), nullable=False),
        StructField('bday', StringType(), nullable=True),
        StructField('chprob', FloatType(), nullable=True),
        StructField('curqa', IntegerType(), nullable=True),
        StructField('blmag', FloatType(), nullable=True),
        StructField('grmag', FloatType(), nullable=True),
        StructField('remag', FloatType(), nullable=True),
        StructField('nimag', FloatType(), nullable=True),
        StructField('s1mag', FloatType(), nullable=True),
        StructField('s2mag', FloatType(), nullable=True),
        StructField('thmag', FloatType(), nullable=True),
        StructField('blrmse', FloatType(), nullable=True),
        StructField('grrmse', FloatType(), nullable=True),
        StructField('rermse', FloatType(), nullable=True),
        StructField('nirmse', FloatType(), nullable=True),
        StructField('s1rmse', FloatType(), nullable=True),
        StructField('s2rmse', FloatType(), nullable=True),
        StructField('thrmse', FloatType(), nullable=True),
        StructField('blcoef', ArrayType(FloatType()), nullable=True),
        StructField('grcoef', ArrayType(FloatType()), nullable=True),
        StructField('recoef', ArrayType(FloatType()), nullable=True),
        StructField('nicoef', ArrayType(FloatType()), nullable=True),
        StructField('s1coef', ArrayType(FloatType()), nullable=True),
        StructField('s2coef', ArrayType(FloatType()), nullable=True),
        StructField('thcoef', ArrayType(FloatType()), nullable=True),
        StructField('blint', FloatType(), nullable=True),
        StructField('grint', FloatType(), nullable=True),
        StructField('reint', FloatType(), nullable=True),
        StructField('niint', FloatType(), nullable=True),
        StructField('s1int', FloatType(), nullable=True),
        StructField('s2int', FloatType(), nullable=True),
        StructField('thint', FloatType(), nullable=True),
        StructField('dates', ArrayType(StringType()), nullable=False),
        StructField('mask', ArrayType(ByteType()), nullable=True),
        StructField('rfrawp', ArrayType(FloatType()), nullable=True),
    ])


def dataframe(ctx, rdd):
    """Creates pyccd dataframe from an rdd of format() rows (pyccd.py:84-96)."""
    require_pyspark('ccdc.pyccd.dataframe')
    from pyspark.sql import SparkSession  # pragma: no cover
    logger(ctx, name=__name__).debug('creating pyccd dataframe...')
    return SparkSession(ctx).createDataFrame(rdd, schema())


def default(change_models):
    """No change models -> one day-1 placeholder row so the pixel is recorded (pyccd.py:99-103)."""
    return [{'start_day': 1, 'end_day': 1, 'break_day': 1}] if not change_models else change_models


def format(cx, cy, px, py, dates, ccdresult):
    """One row dict per change model (pyccd.py:106-148).  ``dates`` in input order, ``mask`` in
    pyccd's sorted-date order, exactly as the reference emits them."""
    rows = [denumpify(
        {'cx': cx,
         'cy': cy,
         'px': px,
         'py': py,
         'sday': date.fromordinal(get('start_day', cm)).isoformat(),
         'eday': date.fromordinal(get('end_day', cm)).isoformat(),
         'bday': date.fromordinal(get('break_day', cm, None)).isoformat(),
         'chprob': get('change_probability', cm, None),
         'curqa': get('curve_qa', cm, None),
         'blmag': get_in(['blue', 'magnitude'], cm, None),
         'grmag': get_in(['green', 'magnitude'], cm, None),
         'remag': get_in(['red', 'magnitude'], cm, None),
         'nimag': get_in(['nir', 'magnitude'], cm, None),
         's1mag': get_in(['swir1', 'magnitude'], cm, None),
         's2mag': get_in(['swir2', 'magnitude'], cm, None),
         'thmag': get_in(['thermal', 'magnitude'], cm, None),
         'blrmse': get_in(['blue', 'rmse'], cm, None),
         'grrmse': get_in(['green', 'rmse'], cm, None),
         'rermse': get_in(['red', 'rmse'], cm, None),
         'nirmse': get_in(['nir', 'rmse'], cm, None),
         's1rmse': get_in(['swir1', 'rmse'], cm, None),
         's2rmse': get_in(['swir2', 'rmse'], cm, None),
         'thrmse': get_in(['thermal', 'rmse'], cm, None),
         'blcoef': get_in(['blue', 'coefficients'], cm, None),
         'grcoef': get_in(['green', 'coefficients'], cm, None),
         'recoef': get_in(['red', 'coefficients'], cm, None),
         'nicoef': get_in(['nir', 'coefficients'], cm, None),
         's1coef': get_in(['swir1', 'coefficients'], cm, None),
         's2coef': get_in(['swir2', 'coefficients'], cm, None),
         'thcoef': get_in(['thermal', 'coefficients'], cm, None),
         'blint': get_in(['blue', 'intercept'], cm, None),
         'grint': get_in(['green', 'intercept'], cm, None),
         'reint': get_in(['red', 'intercept'], cm, None),
         'niint': get_in(['nir', 'intercept'], cm, None),
         's1int': get_in(['swir1', 'intercept'], cm, None),
         's2int': get_in(['swir2', 'intercept'], cm, None),
         'thint': get_in(['thermal', 'intercept'], cm, None),
         'dates': None,  # (set below: built here, native already)
         'mask': get('processing_mask', ccdresult, None)})
        for cm in default(get('change_models', ccdresult, None))]
    for row in rows:
        row['dates'] = _iso_dates(dates)
    return rows


def detect(timeseries):
    """Takes in a timeseries ((cx, cy, px, py), {dates, blues..thermals, qas}) and returns a list
    of detections (pyccd.py:151-168)."""
    cx, cy, px, py = first(timeseries)
    return format(cx=cx,
                  cy=cy,
                  px=px,
                  py=py,
                  dates=get('dates', second(timeseries)),
                  ccdresult=ccd.detect(**second(timeseries)))


def detect_partition(records, params=None):
    """Batched detect over an iterable of timeseries records: pixels sharing a date vector go
    to the GPU in one call; rows come out in record order, identical to ``detect``."""
    records = list(records)
    rows = []
    for (key, res), (_, rec) in zip(ccd.detect_records(records, params), records):
        cx, cy, px, py = key
        rows.extend(format(cx=cx, cy=cy, px=px, py=py, dates=get('dates', rec), ccdresult=res))
    return rows


def _run_chips(chips, params, context, symmetric=True):
    """Group chipmunk chips by location, batch locations that share a date vector, stage each
    batch with the device chip packer and detect it.  Yields (ctx, chip index, (cx, cy),
    dates [n] int64 descending, n_pix) for every location, batch by batch.  symmetric=False
    accepts locations whose layers lack some dates (they stage as fill, QA 1) instead of
    raising like merlin's symmetric date check."""
    import ccdgpu
    from ccdc import chipmunk
    groups = chipmunk.group(chips)
    ctx = context or ccdgpu.default_context()
    batches = {}
    for key, layers in groups.items():
        d = chipmunk.dates_of(layers, symmetric)
        batches.setdefault(d.tobytes(), []).append((key, layers))
    for members in batches.values():
        dates, text, offsets = chipmunk.pack_text([layers for _, layers in members], symmetric)
        first_payload = next(v for _, layers in members for n in chipmunk.LAYERS for v in layers[n].values())
        n_pix = chipmunk.payload_pixels(first_payload)
        ctx.stage_chipmunk(dates, text, offsets, n_pix, params)
        ctx.run()
        for c, (key, _) in enumerate(members):
            yield ctx, c, key, dates[0], n_pix


def detect_chips(chips, params=None, context=None, symmetric=True):
    """Change detection straight from chipmunk chips (the wire format merlin.create consumes in
    timeseries.rdd, timeseries.py:120): chips of any number of locations, grouped by location,
    batched by shared date vector, decoded and pivoted on the device (ccdc.chipmunk,
    ccdgpu.Context.stage_chipmunk) and detected there.  Returns the rows ``detect`` would give
    for every pixel of every location (pixel keys as test/__init__.py:37: px = cx + 30 col,
    py = cy - 30 row), locations in first-seen order.  Raises ValueError (QAValueError) on an
    unsupported QA value, like ccd.detect.  symmetric: see _run_chips."""
    import ccdgpu
    from ccdgpu import abi
    from ccdc import timeseries
    rows = {}
    order = []
    for ctx, c, (cx, cy), dates, n_pix in _run_chips(chips, params, context, symmetric):
        u = ctx.fetch(c)
        if u.error_pixel >= 0:
            raise ccdgpu.QAValueError('unsupported QA value at pixel %d of chip (%d, %d)' % (u.error_pixel, cx, cy))
        dlist = [int(x) for x in dates]
        out = []
        for px, (_, _, ppx, ppy) in enumerate(timeseries.chip_keys(cx, cy, n_pix)):
            out.extend(format(cx=cx, cy=cy, px=ppx, py=ppy, dates=dlist,
                              ccdresult=abi.pixel_result(u, px, ccd.algorithm)))
        rows[(cx, cy)] = out
        order.append((cx, cy))
    return [r for key in order for r in rows[key]]


def detect_chips_tables(chips, params=None, context=None, width=100):
    """Columnar variant of ``detect_chips``: [((cx, cy), {'segment', 'pixel', 'chip'} Arrow
    tables)] with the reference's column names and storage types (ccdc.sink), the rows packed
    on the device (ccdgpu.Context.fetch_rows) instead of formatted one dict at a time."""
    import ccdgpu
    from ccdc import sink
    out = []
    for ctx, c, (cx, cy), dates, n_pix in _run_chips(chips, params, context):
        u = ctx.fetch(c)  # procedure / QA error check
        if u.error_pixel >= 0:
            raise ccdgpu.QAValueError('unsupported QA value at pixel %d of chip (%d, %d)' % (u.error_pixel, cx, cy))
        off, rows, mask = ctx.fetch_rows(c, cx, cy, width)
        out.append(((cx, cy), sink.tables(cx, cy, dates, off, rows, mask)))
    return out


def rdd(ctx, timeseries):
    """Run change detection against an RDD of timeseries (pyccd.py:171-183)."""
    logger(context=ctx, name=__name__).info('executing change detection...')
    return timeseries.mapPartitions(detect_partition)
