"""The tile driver on the GPU (ccdc.runner.changedetection; reference core.changedetection,
ccdc/core.py:78-123): chips of the reference tile grid (test/data/tile_response.json) with
synthetic ARD of both cadences, two contexts per GPU with pinned uploads in the transport
encoding, device row packing, per-chip rows gathered -- checked against rows restated from the C
oracle, and byte-identical however the chips are batched, whether they are uploaded encoded or
raw and whether the contexts reserve CUs for their uploads."""
import json
import os

import numpy as np
import pytest

import oracle_ctypes
from rows_util import rows_from_result

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_PIX = 300
N_CHIPS = 8


def tile():
    with open(os.path.join(ROOT, 'tests', 'golden', 'chipmunk', 'tile_response.json')) as f:
        return json.load(f)


def chip(p):
    from ccdgpu import synth
    return synth.chip(synth.config(5 if p % 3 == 2 else 3), p, 0, N_PIX)


def source(pos):
    import ccdgpu
    return ccdgpu.ChipBatch.from_chips([chip(p) for p in pos], pinned=True)


def run(contexts, batch_chips, encode=True, copy_cus=8):
    from ccdc import runner
    sink = runner.SummarySink(keep_rows=True)
    res = runner.changedetection(tile(), source, device=0, contexts=contexts, batch_chips=batch_chips,
                                 number=N_CHIPS, sink=sink, encode=encode, copy_cus=copy_cus)
    return res, sink


def test_tile_runner_rows_match_oracle_and_batching():
    res, sink = run(2, 3)
    t = tile()
    assert res['xys'] == tuple((int(x), int(y)) for x, y in t['chips'][:N_CHIPS])
    assert {c['n_obs'] for c in res['chips']} == {1421, 2121}
    for p in range(N_CHIPS):
        d, s, q = chip(p)
        rc, u = oracle_ctypes.detect_batch(d, s, q, threads=16)
        assert rc == 0
        cx, cy = (int(v) for v in t['chips'][p])
        ro, rr = rows_from_result(u, cx, cy)
        off, rows, mask = sink.rows[p]
        assert np.array_equal(off, ro), p
        for f in ('px', 'py', 'sday', 'eday', 'bday', 'curqa', 'has_model'):
            assert np.array_equal(rows[f], rr[f]), (p, f)
        for f in ('chprob', 'mag', 'rmse', 'intercept', 'coef'):
            np.testing.assert_allclose(rows[f], rr[f], rtol=1e-6, atol=1e-6, err_msg='%d %s' % (p, f))
        assert np.array_equal(mask, u.mask.astype(np.int8)), p
    res2, _ = run(1, 5)
    assert [c['digest'] for c in res2['chips']] == [c['digest'] for c in res['chips']]
    # the runner's default upload is the transport encoding: raw uploads give the same rows
    res3, _ = run(2, 4, encode=False)
    assert [c['digest'] for c in res3['chips']] == [c['digest'] for c in res['chips']]
    # and so do contexts without CUs reserved for the upload stream (ccdgpu_init_copy_cus)
    res4, _ = run(2, 3, copy_cus=0)
    assert [c['digest'] for c in res4['chips']] == [c['digest'] for c in res['chips']]
