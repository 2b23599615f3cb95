"""Classification features on the HIP path: the segment table the device
writes for a chip (pyccd.detect_chips_tables: device detection + device row packing) joined with
an aux table into the random forest's feature matrix (features.dataframe / matrix, reference
features.py + udfs.densify), against the same pipeline over rows restated from the C oracle's
results for the same chip."""
import numpy as np
import pyarrow as pa
import pytest

import oracle_ctypes
from rows_util import rows_from_result

CX, CY = -1815585, 1064805


def _aux(n_pix, width=100, seed=3):
    rng = np.random.default_rng(seed)
    p = np.arange(n_pix)
    return pa.table({'cx': pa.array(np.full(n_pix, CX, np.int32)),
                     'cy': pa.array(np.full(n_pix, CY, np.int32)),
                     'px': pa.array((CX + 30 * (p % width)).astype(np.int32)),
                     'py': pa.array((CY - 30 * (p // width)).astype(np.int32)),
                     'dem': pa.array([[float(x)] for x in rng.normal(size=n_pix)], type=pa.list_(pa.float32())),
                     'trends': pa.array([[int(x)] for x in rng.integers(0, 9, n_pix)], type=pa.list_(pa.int32())),
                     'aspect': pa.array([[int(x)] for x in rng.integers(0, 360, n_pix)], type=pa.list_(pa.int32())),
                     'posidex': pa.array([[float(x)] for x in rng.random(n_pix)], type=pa.list_(pa.float32())),
                     'slope': pa.array([[float(x)] for x in rng.random(n_pix)], type=pa.list_(pa.float32())),
                     'mpw': pa.array([[int(x)] for x in rng.integers(0, 100, n_pix)], type=pa.list_(pa.int32()))})


@pytest.mark.gpu
def test_features_from_device_rows_match_oracle_rows():
    from ccdc import chipmunk, features, pyccd, sink
    from ccdgpu import synth
    n_pix = 300
    d, s, q = synth.chip(synth.config(5), 4, 0, n_pix)
    order = np.argsort(d)[::-1]  # chipmunk's newest-first order
    d, s, q = d[order], s[:, :, order], q[:, order]
    (key, t), = pyccd.detect_chips_tables(chipmunk.chip_response(CX, CY, d, s, q))
    got_seg = t['segment']
    rc, u = oracle_ctypes.detect_batch(d, s, q, threads=16)
    assert rc == 0
    _, rows = rows_from_result(u, CX, CY)
    ref_seg = sink.segment_table(CX, CY, rows)
    assert got_seg.num_rows == ref_seg.num_rows > n_pix
    aux = _aux(n_pix)
    gt, rt = features.dataframe(aux, got_seg), features.dataframe(aux, ref_seg)
    assert gt.num_rows == rt.num_rows == got_seg.num_rows
    for c in ('cx', 'cy', 'px', 'py', 'sday', 'eday', 'label'):
        assert gt[c].to_pylist() == rt[c].to_pylist(), c
    gm, rm = features.matrix(gt), features.matrix(rt)
    assert gm.shape == rm.shape == (gt.num_rows, 33)
    # float32 row values of two FP64 results that agree to ~1e-9: equal up to one float32 rounding
    np.testing.assert_array_equal(np.isnan(gm), np.isnan(rm))
    np.testing.assert_allclose(gm, rm, rtol=1e-6, atol=1e-6, equal_nan=True)
