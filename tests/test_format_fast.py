"""ccdc.pyccd.format's fast paths (ISO date strings built once per date vector, native lists
copied in one pass by denumpify, the mask as Python ints from one numpy conversion) give the rows
of the reference's literal per-row code (pyccd.py:106-148 with merlin's denumpify) -- same values,
same types, same key order -- on change-dense multi-segment pixels (C oracle results, CPU)."""
import os
import sys
from datetime import date

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(ROOT, 'lcmap-firebird_amd'), os.path.join(ROOT, 'oracle')]

import ccd  # noqa: E402
import oracle_ctypes  # noqa: E402
from ccdc import pyccd  # noqa: E402
from ccdgpu import abi, synth  # noqa: E402


def _literal_denumpify(arg):
    if isinstance(arg, np.generic):
        return arg.item()
    if isinstance(arg, np.ndarray):
        return arg.tolist()
    if isinstance(arg, dict):
        return {k: _literal_denumpify(v) for k, v in arg.items()}
    if isinstance(arg, list):
        return [_literal_denumpify(v) for v in arg]
    if isinstance(arg, tuple):
        return tuple(_literal_denumpify(v) for v in arg)
    return arg


def _literal_rows(cx, cy, px, py, dates, res):
    g, gi = pyccd.get, pyccd.get_in
    rows = []
    for cm in pyccd.default(g('change_models', res, None)):
        row = {'cx': cx, 'cy': cy, 'px': px, 'py': py,
               'sday': date.fromordinal(g('start_day', cm)).isoformat(),
               'eday': date.fromordinal(g('end_day', cm)).isoformat(),
               'bday': date.fromordinal(g('break_day', cm, None)).isoformat(),
               'chprob': g('change_probability', cm, None), 'curqa': g('curve_qa', cm, None)}
        for what, suffix in (('magnitude', 'mag'), ('rmse', 'rmse'), ('coefficients', 'coef'), ('intercept', 'int')):
            for band, pre in zip(abi.BANDS, ('bl', 'gr', 're', 'ni', 's1', 's2', 'th')):
                row[pre + suffix] = gi([band, what], cm, None)
        row['dates'] = [date.fromordinal(o).isoformat() for o in dates]
        row['mask'] = g('processing_mask', res, None)
        rows.append(_literal_denumpify(row))
    return rows


def test_format_rows_equal_the_literal_restatement():
    d, s, q = synth.chip(synth.config(5), 3, 0, 40)
    rc, u = oracle_ctypes.detect_batch(d, s, q, threads=4)
    assert rc == 0
    dl = [int(x) for x in d]
    n_rows = 0
    for p in range(q.shape[0]):
        a, b = int(u.seg_offsets[p]), int(u.seg_offsets[p + 1])
        literal_res = {'processing_mask': [int(x) for x in u.mask[p]],
                       'change_models': [abi.segment_to_change_model(x) for x in u.segments[a:b]]}
        got = pyccd.format(cx=1, cy=2, px=3 + p, py=4, dates=dl, ccdresult=abi.pixel_result(u, p, ccd.algorithm))
        want = _literal_rows(1, 2, 3 + p, 4, dl, literal_res)
        assert len(got) == len(want)
        for x, y in zip(got, want):
            assert list(x) == [k for k in list(y) if k in x] and set(x) == set(y)
            for k in y:
                assert x[k] == y[k] and type(x[k]) is type(y[k]), k
                if isinstance(y[k], (list, tuple)):
                    assert [type(v) for v in x[k]] == [type(v) for v in y[k]], k
        n_rows += len(got)
    assert n_rows > 3 * q.shape[0]  # change-dense: several segments per pixel


def test_denumpify_fast_path_keeps_numpy_conversion():
    mixed = [1, np.int64(2), 3.0, np.float32(4.5), None, 'x', True]
    out = pyccd.denumpify({'a': mixed, 'b': tuple(mixed), 'c': [1, 2, 3]})
    assert out == {'a': [1, 2, 3.0, 4.5, None, 'x', True], 'b': (1, 2, 3.0, 4.5, None, 'x', True), 'c': [1, 2, 3]}
    assert [type(v) for v in out['a']] == [int, int, float, float, type(None), str, bool]
    lst = [5, 6]
    assert pyccd.denumpify(lst) is not lst  # a copy, as the recursive form made


def test_iso_dates_of_an_iterator_and_a_numpy_vector():
    d = np.array([734973, 731205, 724404], dtype=np.int64)
    want = ['2013-04-15', '2002-12-21', '1984-05-08']
    assert pyccd._iso_dates(d) == want
    assert pyccd._iso_dates(iter([734973, 731205, 724404])) == want
    a = pyccd._iso_dates([734973, 731205, 724404])
    a.append('x')  # a new list per call
    assert pyccd._iso_dates([734973, 731205, 724404]) == want
