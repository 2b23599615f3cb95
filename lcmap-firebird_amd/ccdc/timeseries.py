"""ccdc.timeseries -- the ARD record layout (mirror of reference ccdc/timeseries.py:23-58) and the
chip packer that turns per-pixel records into the band-major, observation-contiguous buffers
the C-ABI consumes (include/ccdgpu.h ccdgpu_detect_batch).  The merlin/chipmunk fetch of
timeseries.rdd (timeseries.py:92-126) is out of scope."""
import numpy as np

from ccdc._types import ArrayType, FloatType, IntegerType, StructField, StructType

BANDS = ('blues', 'greens', 'reds', 'nirs', 'swir1s', 'swir2s', 'thermals')


def schema(name):
    """Return Dataframe schema for named timeseries (timeseries.py:23-58)."""
    s = {'ard': StructType([StructField('cx', IntegerType(), nullable=False),
                            StructField('cy', IntegerType(), nullable=False),
                            StructField('px', IntegerType(), nullable=False),
                            StructField('py', IntegerType(), nullable=False),
                            StructField('dates', ArrayType(IntegerType(), False), nullable=False),
                            StructField('blues', ArrayType(IntegerType(), False), nullable=False),
                            StructField('greens', ArrayType(IntegerType(), False), nullable=False),
                            StructField('reds', ArrayType(IntegerType(), False), nullable=False),
                            StructField('nirs', ArrayType(IntegerType(), False), nullable=False),
                            StructField('swir1s', ArrayType(IntegerType(), False), nullable=False),
                            StructField('swir2s', ArrayType(IntegerType(), False), nullable=False),
                            StructField('thermals', ArrayType(IntegerType(), False), nullable=False),
                            StructField('qas', ArrayType(IntegerType(), False), nullable=False)]),
         'aux': StructType([StructField('cx', IntegerType(), nullable=False),
                            StructField('cy', IntegerType(), nullable=False),
                            StructField('px', IntegerType(), nullable=False),
                            StructField('py', IntegerType(), nullable=False),
                            StructField('dates', ArrayType(IntegerType(), False), nullable=False),
                            StructField('dem', ArrayType(FloatType(), False), nullable=True),
                            StructField('trends', ArrayType(IntegerType(), False), nullable=False),
                            StructField('aspect', ArrayType(IntegerType(), False), nullable=True),
                            StructField('posidex', ArrayType(FloatType(), False), nullable=True),
                            StructField('slope', ArrayType(FloatType(), False), nullable=True),
                            StructField('mpw', ArrayType(IntegerType(), False), nullable=True)])}
    return s.get(name) if name else s


def pack(records):
    """Per-pixel ard records [((cx,cy,px,py), {dates, blues..thermals, qas}), ...] that share one
    date vector -> (keys, dates[n] int64, spectra[7][n_pix][n] int16, qa[n_pix][n] uint16)."""
    records = list(records)
    keys = [k for k, _ in records]
    dates = np.asarray(records[0][1]['dates'], dtype=np.int64)
    n = dates.shape[0]
    spectra = np.empty((7, len(records), n), dtype=np.int16)
    qa = np.empty((len(records), n), dtype=np.uint16)
    for j, (_, rec) in enumerate(records):
        if not np.array_equal(np.asarray(rec['dates'], dtype=np.int64), dates):
            raise ValueError('pack() needs records that share one date vector (one chip)')
        for b, name in enumerate(BANDS):
            spectra[b, j] = rec[name]
        qa[j] = rec['qas']
    return keys, dates, spectra, qa


def unpack(keys, dates, spectra, qa):
    """Inverse of pack(): the per-pixel records merlin.create would have produced."""
    out = []
    d = [int(x) for x in dates]
    for j, key in enumerate(keys):
        rec = {name: spectra[b, j].copy() for b, name in enumerate(BANDS)}
        rec['qas'] = qa[j].copy()
        rec['dates'] = list(d)
        out.append((tuple(key), rec))
    return out


def chip_keys(cx, cy, n_pix=10000, width=100):
    """(cx, cy, px, py) keys of a chip's pixels in row-major order (30 m pixels; reference test
    element test/__init__.py:37 has px = cx + 30*col, py = cy - 30*row)."""
    return [(cx, cy, cx + 30 * (i % width), cy - 30 * (i // width)) for i in range(n_pix)]
