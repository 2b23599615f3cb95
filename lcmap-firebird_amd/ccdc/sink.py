"""ccdc.sink -- columnar output of the detection results.

The reference turns every change model into a Python row dict (ccdc/pyccd.py:106-148), lets
Spark cast it to the ccd dataframe schema (pyccd.py:39-81, float64 -> FloatType) and writes the
projections ``segment`` / ``pixel`` / ``chip`` (segment.py:16-55, pixel.py, chip.py) to
Cassandra (resources/schema.cql).  Here the rows come off the device already in their storage
types (``ccdgpu.Context.fetch_rows``: float32, one byte per mask entry, ccd_rows.hip) and are
assembled column-wise into Arrow tables whose column names and types follow the reference
schemas exactly; ``write_parquet`` is the offline sink (the Cassandra writer stays out of scope,
SURVEY.md §2).  A pixel without change models keeps pyccd.default's day-1 row with every band,
chprob and curqa column null, as in the reference.  A model with break_day 0 (the single fit of
the permanent-snow and insufficient-clear procedures) is written with a null bday -- the one
deliberate difference: the reference's format raises ValueError on that row.
"""
import os

import numpy as np
import pyarrow as pa

from ccdc import _types
from ccdc import chip as chip_mod
from ccdc import pixel as pixel_mod
from ccdc import pyccd as pyccd_mod
from ccdc import segment as segment_mod

BAND_PREFIX = ('bl', 'gr', 're', 'ni', 's1', 's2', 'th')

_EPOCH = np.datetime64('0001-01-01', 'D')


def arrow_type(t):
    """Spark SQL type (ccdc._types / pyspark) -> Arrow type with the same storage width."""
    if isinstance(t, _types.ArrayType):
        return pa.list_(arrow_type(t.elementType))
    return {'int': pa.int32(), 'float': pa.float32(), 'string': pa.string(), 'tinyint': pa.int8(),
            'timestamp': pa.timestamp('us')}[t.simpleString()]


def arrow_schema(spark_schema):
    return pa.schema([pa.field(f.name, arrow_type(f.dataType), nullable=f.nullable) for f in spark_schema])


def iso_days(ordinals):
    """Proleptic ordinals -> 'YYYY-MM-DD' strings (date.fromordinal(o).isoformat(), vectorised)."""
    o = np.asarray(ordinals, dtype=np.int64)
    return (_EPOCH + (o - 1).astype('timedelta64[D]')).astype('datetime64[D]').astype(str)


def _float_col(values, valid):
    return pa.array(values.astype(np.float32), type=pa.float32(), mask=~valid)


def _list_col(values, valid):
    """[n][k] float32 -> list<float32> column, null where not valid."""
    v = np.ascontiguousarray(values, dtype=np.float32)
    n, k = v.shape
    offsets = pa.array(np.arange(0, (n + 1) * k, k, dtype=np.int32))
    lst = pa.ListArray.from_arrays(offsets, pa.array(v.reshape(-1), type=pa.float32()),
                                   mask=pa.array(~valid))
    return lst


def _row_columns(cx, cy, rows):
    """Columns shared by the ccd and segment tables (pyccd.format keys, pyccd.py:106-145)."""
    n = rows.shape[0]
    valid = rows['has_model'] != 0
    cols = {
        'cx': pa.array(np.full(n, cx, np.int32)), 'cy': pa.array(np.full(n, cy, np.int32)),
        'px': pa.array(rows['px']), 'py': pa.array(rows['py']),
        'sday': pa.array(iso_days(rows['sday'])), 'eday': pa.array(iso_days(rows['eday'])),
        # break_day 0 (permanent-snow / insufficient-clear models have no break): null bday.
        # The reference's pyccd.format would raise in date.fromordinal(0) on such a row
        # (SURVEY.md §7 edge (a)); the bday column is nullable in its schema (pyccd.py:46).
        'bday': pa.array(iso_days(np.maximum(rows['bday'], 1)), mask=rows['bday'] < 1),
        'chprob': _float_col(rows['chprob'], valid),
        'curqa': pa.array(rows['curqa'].astype(np.int32), mask=~valid),
    }
    for b, pre in enumerate(BAND_PREFIX):
        cols[pre + 'mag'] = _float_col(rows['mag'][:, b], valid)
        cols[pre + 'rmse'] = _float_col(rows['rmse'][:, b], valid)
        cols[pre + 'coef'] = _list_col(rows['coef'][:, b, :], valid)
        cols[pre + 'int'] = _float_col(rows['intercept'][:, b], valid)
    cols['rfrawp'] = pa.nulls(n, type=pa.list_(pa.float32()))
    return cols


def _fixed_lists(values, n_lists, typ):
    """n_lists equal-length lists from a flat value array."""
    k = len(values) // n_lists if n_lists else 0
    offsets = pa.array(np.arange(0, (n_lists + 1) * k, k if k else 1, dtype=np.int32)[:n_lists + 1])
    return pa.ListArray.from_arrays(offsets, pa.array(values, type=typ))


def _build(spark_schema, cols):
    schema = arrow_schema(spark_schema)
    return pa.table([cols[f.name] for f in schema], schema=schema)


def segment_table(cx, cy, rows):
    """segment table (segment.schema(), segment.py:16-55): one row per change model."""
    return _build(segment_mod.schema(), _row_columns(cx, cy, rows))


def pixel_table(cx, cy, row_offsets, rows, mask):
    """pixel table (pixel.schema()): cx, cy, px, py, processing mask (sorted order, 0/1)."""
    first = np.asarray(row_offsets[:-1])
    m = np.asarray(mask, dtype=np.int8)
    n = m.shape[0]
    cols = {'cx': pa.array(np.full(n, cx, np.int32)), 'cy': pa.array(np.full(n, cy, np.int32)),
            'px': pa.array(rows['px'][first]), 'py': pa.array(rows['py'][first]),
            'mask': _fixed_lists(m.reshape(-1), n, pa.int8())}
    return _build(pixel_mod.schema(), cols)


def chip_table(cx, cy, dates):
    """chip table (chip.schema()): the chip's acquisition dates, input order, ISO text."""
    cols = {'cx': pa.array([cx], type=pa.int32()), 'cy': pa.array([cy], type=pa.int32()),
            'dates': pa.array([iso_days(dates).tolist()], type=pa.list_(pa.string()))}
    return _build(chip_mod.schema(), cols)


def ccd_table(cx, cy, dates, row_offsets, rows, mask):
    """The full ccd dataframe of one chip (pyccd.schema(), pyccd.py:39-81), every row carrying
    the chip's dates and its pixel's mask as pyccd.format does (heavy: n_rows x n_obs)."""
    n = rows.shape[0]
    cols = _row_columns(cx, cy, rows)
    pix_of_row = np.repeat(np.arange(len(row_offsets) - 1), np.diff(row_offsets))
    iso = iso_days(dates)
    cols['dates'] = _fixed_lists(np.tile(iso, n), n, pa.string())
    cols['mask'] = _fixed_lists(np.asarray(mask, dtype=np.int8)[pix_of_row].reshape(-1), n, pa.int8())
    return _build(pyccd_mod.schema(), cols)


def tables(cx, cy, dates, row_offsets, rows, mask):
    """{'segment', 'pixel', 'chip'} Arrow tables of one chip (the reference's Cassandra tables)."""
    return {'segment': segment_table(cx, cy, rows),
            'pixel': pixel_table(cx, cy, row_offsets, rows, mask),
            'chip': chip_table(cx, cy, dates)}


def write_parquet(directory, chip_tables, cx, cy, **options):
    """Offline sink: <directory>/<table>/<cx>_<cy>.parquet per table.  ``options`` go to
    pyarrow.parquet.write_table (e.g. use_dictionary=False: the pixel table's mask in about half
    the time, at ~8x the file size)."""
    import pyarrow.parquet as pq
    paths = {}
    for name, t in chip_tables.items():
        d = os.path.join(directory, name)
        os.makedirs(d, exist_ok=True)
        paths[name] = os.path.join(d, '%d_%d.parquet' % (cx, cy))
        pq.write_table(t, paths[name], **options)
    return paths
