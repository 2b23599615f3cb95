"""Classification features: the reference's column contract
(test/test_features.py) and the column-wise feature matrix against a per-row restatement of
udfs.densify over the joined rows."""
import numpy as np
import pyarrow as pa

from ccdc import features, sink
from ccdgpu import abi

# reference test/__init__.py:22-30
AUXBASE = ['aspect', 'dem', 'mpw', 'posidex', 'slope']
ATTRBASE = ['blmag', 'grmag', 'remag', 'nimag', 's1mag', 's2mag', 'thmag', 'blrmse',
            'grrmse', 'rermse', 'nirmse', 's1rmse', 's2rmse', 'thrmse', 'blcoef', 'grcoef',
            'recoef', 'nicoef', 's1coef', 's2coef', 'thcoef', 'blint', 'grint', 'reint',
            'niint', 's1int', 's2int', 'thint']


def test_columns():
    assert set(features.columns()) == set(ATTRBASE + AUXBASE + ['grint'])
    assert len(features.columns()) == 33 and features.columns()[-5:] == ['dem', 'aspect', 'slope', 'mpw', 'posidex']


def _tables(seed=0, n_pix=6):
    rng = np.random.default_rng(seed)
    nrow = [1, 3, 1, 2, 1, 2][:n_pix]
    rows = np.zeros(sum(nrow), abi.ROW_DTYPE)
    off = np.concatenate([[0], np.cumsum(nrow)])
    for p in range(n_pix):
        rows['px'][off[p]:off[p + 1]] = 30 * p
    rows['sday'] = rng.integers(723000, 735000, len(rows))
    rows['eday'] = rows['sday'] + 400
    rows['bday'] = rows['eday'] + 10
    rows['has_model'] = 1
    rows['has_model'][0] = 0  # a default row (null band columns)
    for f in ('mag', 'rmse', 'intercept'):
        rows[f] = rng.normal(size=rows[f].shape).astype(np.float32)
    rows['coef'] = rng.normal(size=rows['coef'].shape).astype(np.float32)
    seg = sink.segment_table(-1815585, 1064805, rows)
    aux = pa.table({'cx': pa.array(np.full(n_pix - 1, -1815585, np.int32)),
                    'cy': pa.array(np.full(n_pix - 1, 1064805, np.int32)),
                    'px': pa.array((30 * np.arange(1, n_pix)).astype(np.int32)),  # pixel 0 has no aux
                    'py': pa.array(np.zeros(n_pix - 1, np.int32)),
                    'dem': pa.array([[float(x), 1.0] for x in rng.normal(size=n_pix - 1)], type=pa.list_(pa.float32())),
                    'trends': pa.array([[int(x), 9] for x in rng.integers(0, 9, n_pix - 1)], type=pa.list_(pa.int32())),
                    'aspect': pa.array([[int(x)] for x in rng.integers(0, 360, n_pix - 1)], type=pa.list_(pa.int32())),
                    'posidex': pa.array([[float(x)] for x in rng.random(n_pix - 1)], type=pa.list_(pa.float32())),
                    'slope': pa.array([[float(x)] for x in rng.random(n_pix - 1)], type=pa.list_(pa.float32())),
                    'mpw': pa.array([[int(x)] for x in rng.integers(0, 100, n_pix - 1)], type=pa.list_(pa.int32()))})
    return seg, aux


def test_dataframe_matches_rowwise_densify():
    seg, aux = _tables()
    t = features.dataframe(aux, seg)
    assert t.column_names == ['cx', 'cy', 'px', 'py', 'sday', 'eday', 'label', 'features']
    got = features.matrix(t)
    joined = features.join({'aux': aux, 'ccd': seg}).to_pylist()
    assert len(joined) == len(got) == seg.num_rows - 1  # the aux-less pixel drops out (inner join)
    want = {(r['px'], r['sday']): features.densify(*[r[c] for c in features.columns()]) for r in joined}
    labels = {(r['px'], r['sday']): r['trends'][0] for r in joined}
    for row, vec in zip(t.to_pylist(), got):
        k = (row['px'], row['sday'])
        np.testing.assert_array_equal(vec, want[k])
        assert row['label'] == labels[k]
    # coefficient columns contribute their first element (the slope); float32 widened exactly
    r0 = joined[0]
    assert want[(r0['px'], r0['sday'])][14] == np.float64(np.float32(r0['blcoef'][0]))


def test_default_rows_give_nan_features():
    seg, aux = _tables()
    aux0 = pa.concat_tables([aux, aux.slice(0, 1).set_column(2, 'px', pa.array([0], type=pa.int32()))])
    t = features.dataframe(aux0, seg)
    m = features.matrix(t)
    px = np.array(t['px'].to_pylist())
    assert np.isnan(m[px == 0][:, :28]).all() and not np.isnan(m[px != 0]).any()
