"""ccdc.features -- classification features over the segment rows (SURVEY.md §8(f) row 4;
mirror of reference ccdc/features.py + ccdc/udfs.py).

The reference joins the aux timeseries with the ccd dataframe on (cx, cy, px, py)
(features.py:6-18), takes ``label = trends[0]`` (features.py:40-50) and packs the 33 columns of
``columns()`` into one dense vector per row with the ``densify`` UDF, which keeps the first
element of list-valued columns (udfs.py:8-22: the slope coefficient of every band's
coefficients, the first aux value) -- the random forest's input (randomforest.py:25-87, out of
scope here).  Here the same steps run column-wise on Arrow tables (ccdc.sink): the feature
matrix is built from whole columns instead of one Python row at a time, with the values Spark
would produce (float32 columns widened to the float64 of Vectors.dense).
"""
import numpy as np
import pyarrow as pa
import pyarrow.compute as pc

KEYS = ['cx', 'cy', 'px', 'py']


def columns():
    """Return list of columns used for generating independent variable (features.py:20-37).
    Order of values is significant: altering it invalidates persisted models."""
    return ['blmag',  'grmag',  'remag',  'nimag',  's1mag',  's2mag',  'thmag',
            'blrmse', 'grrmse', 'rermse', 'nirmse', 's1rmse', 's2rmse', 'thrmse',
            'blcoef', 'grcoef', 'recoef', 'nicoef', 's1coef', 's2coef', 'thcoef',
            'blint',  'grint',  'reint',  'niint',  's1int',  's2int',  'thint',
            'dem',    'aspect', 'slope',  'mpw',    'posidex']


def densify(*args, **kwargs):
    """udfs.densify for one row: first element of list-like values, the value otherwise ->
    a float64 vector (pyspark.ml.linalg.Vectors.dense)."""
    fn = lambda x: next(iter(x)) if type(x) in (tuple, set, list) else x
    return np.array([np.nan if v is None else float(v) for v in map(fn, args)], dtype=np.float64)


def join(dfs):
    """Join aux and ccd tables on the pixel key (features.py:6-18), inner: the keys once, then
    the aux and ccd columns (Arrow's hash join runs on the keys and row numbers only, so
    list-valued columns of either side come along by ``take``)."""
    aux, ccd = dfs['aux'], dfs['ccd']
    a = aux.select(KEYS).append_column('_a', pa.array(np.arange(aux.num_rows, dtype=np.int64)))
    c = ccd.select(KEYS).append_column('_c', pa.array(np.arange(ccd.num_rows, dtype=np.int64)))
    j = a.join(c, keys=KEYS, join_type='inner').sort_by([('_c', 'ascending')])
    at, ct = aux.take(j['_a']), ccd.take(j['_c'])
    cols = {k: ct[k] for k in KEYS}
    cols.update({n: at[n] for n in aux.column_names if n not in KEYS})
    cols.update({n: ct[n] for n in ccd.column_names if n not in KEYS and n not in cols})
    return pa.table(cols)


def dependent(table):
    """label = trends[0] (features.py:40-50)."""
    label = pc.list_element(table['trends'], 0)
    return table.append_column('label', label)


def _first(col):
    """Column -> float64 numpy array: list columns by their first element, nulls as NaN."""
    if pa.types.is_list(col.type) or pa.types.is_large_list(col.type):
        col = pc.list_element(col, 0)
    return pc.cast(col, pa.float64()).to_numpy(zero_copy_only=False)


def independent(table):
    """features = densify(*columns()) per row (features.py:53-63), built column-wise: a
    fixed-size list<double>[33] column."""
    mat = np.stack([_first(table[name]) for name in columns()], axis=1)
    flat = pa.array(mat.reshape(-1), type=pa.float64())
    return table.append_column('features', pa.FixedSizeListArray.from_arrays(flat, len(columns())))


def dataframe(aux, ccd):
    """Training / classification table: location, label and features (features.py:66-83)."""
    t = independent(dependent(join({'aux': aux, 'ccd': ccd})))
    return t.select(['cx', 'cy', 'px', 'py', 'sday', 'eday', 'label', 'features'])


def matrix(table):
    """The features column of ``independent`` / ``dataframe`` as a float64 [n_rows][33] array."""
    col = table['features'].combine_chunks()
    return col.flatten().to_numpy(zero_copy_only=False).reshape(-1, len(columns()))
