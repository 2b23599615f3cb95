"""The reference's own boundary tests for the hot path, re-stated against the mirror package
(reference test/test_pyccd.py:18-132, test_segment.py:50-56, test_pixel.py:8-14,
test_chip.py:8-14, test_timeseries.py:14-25), plus the implied known answer of test_detect
(the all-fill 4-observation element) through the oracle.  CPU only: the GPU-backed run of
test_detect is in tests/test_gpu.py."""
import datetime

import numpy as np
import pytest

import ccd_ref
from ccdc import chip, pixel, pyccd, segment, timeseries

# test/__init__.py:21-34 key lists (data)
SCHEMABASE = ['cx', 'cy', 'px', 'py', 'dates']
ATTRBASE = ['blmag', 'grmag', 'remag', 'nimag', 's1mag', 's2mag', 'thmag', 'blrmse',
            'grrmse', 'rermse', 'nirmse', 's1rmse', 's2rmse', 'thrmse', 'blcoef', 'grcoef',
            'recoef', 'nicoef', 's1coef', 's2coef', 'thcoef', 'blint', 'grint', 'reint',
            'niint', 's1int', 's2int', 'thint']
CCD_SCHEMA_BASE = SCHEMABASE + ATTRBASE + ['sday', 'eday', 'bday', 'chprob', 'curqa', 'mask']
CCD_FORMAT_KEYS = CCD_SCHEMA_BASE + ['grint']
CCD_SCHEMA_NAMES = CCD_SCHEMA_BASE + ['rfrawp']

# test/__init__.py:37-46
TIMESERIES_ELEMENT = ((-1815585, 1064805, -1814475, 1062105),
                      {'blues': np.array([-9999] * 4, dtype=np.int16),
                       'qas': np.array([1, 1, 1, 1], dtype=np.uint16),
                       'nirs': np.array([-9999] * 4, dtype=np.int16),
                       'thermals': np.array([-9999] * 4, dtype=np.int16),
                       'swir2s': np.array([-9999] * 4, dtype=np.int16),
                       'reds': np.array([-9999] * 4, dtype=np.int16),
                       'swir1s': np.array([-9999] * 4, dtype=np.int16),
                       'greens': np.array([-9999] * 4, dtype=np.int16),
                       'dates': [734973, 731205, 724404, 723868]})


def test_algorithm():
    assert 'lcmap-pyccd' in pyccd.algorithm()


def test_table():
    assert 'data' == pyccd.table()


def test_schema():
    assert set(pyccd.schema().names) == set(CCD_SCHEMA_NAMES)


def test_default():
    assert pyccd.default([]) == [{'start_day': 1, 'end_day': 1, 'break_day': 1}]
    assert pyccd.default(['foo', 'bar']) == ['foo', 'bar']


def test_format():
    """test_pyccd.py:37-126 golden dict."""
    chipx, chipy, pixelx, pixely = 100, -100, 50, -50
    sday, eday, bday = 1, 3, 2
    sdate = datetime.date.fromordinal(sday).isoformat()
    edate = datetime.date.fromordinal(eday).isoformat()
    bdate = datetime.date.fromordinal(bday).isoformat()
    fval = 0.5
    model = {'magnitude': fval, 'rmse': fval, 'coefficients': (fval, fval), 'intercept': fval}
    cm = {'start_day': sday, 'end_day': eday, 'break_day': bday, 'observation_count': 3,
          'change_probability': fval, 'curve_qa': fval}
    for b in ('blue', 'green', 'red', 'nir', 'swir1', 'swir2', 'thermal'):
        cm[b] = model
    expected = {'cx': chipx, 'cy': chipy, 'px': pixelx, 'py': pixely,
                'sday': sdate, 'eday': edate, 'bday': bdate, 'chprob': fval, 'curqa': fval,
                'dates': [sdate, bdate, edate], 'mask': [0, 1, 0]}
    for pre in ('bl', 'gr', 're', 'ni', 's1', 's2', 'th'):
        expected[pre + 'mag'] = fval
        expected[pre + ('rmse' if pre != 'ni' else 'rmse')] = fval
        expected[pre + 'coef'] = (fval, fval)
        expected[pre + 'int'] = fval
    out = pyccd.format(cx=chipx, cy=chipy, px=pixelx, py=pixely, dates=[sday, bday, eday],
                       ccdresult={'processing_mask': [0, 1, 0], 'change_models': [cm]})
    assert out[0] == expected


def test_detect_fill_element_known_answer(monkeypatch):
    """test_pyccd.py:129-132 through the format plumbing, with ccd.detect answered by the
    numpy restatement (the GPU-backed version of this test is tests/test_gpu.py)."""
    import ccd
    monkeypatch.setattr(ccd, 'detect', ccd_ref.detect)
    rows = pyccd.detect(TIMESERIES_ELEMENT)
    assert len(rows) == 1
    r = rows[0]
    assert r['cx'] == -1815585
    assert set(r.keys()) == set(CCD_FORMAT_KEYS)
    assert r['sday'] == r['eday'] == r['bday'] == '0001-01-01'
    assert r['dates'] == ['2013-04-15', '2002-12-21', '1984-05-08', '1982-11-19']
    assert r['mask'] == [0, 0, 0, 0]
    assert all(r[k] is None for k in ATTRBASE + ['chprob', 'curqa'])


def test_segment_schema():
    assert segment.table() == 'segment'
    assert segment.schema().simpleString() == (
        'struct<cx:int,cy:int,px:int,py:int,sday:string,eday:string,bday:string,chprob:float,'
        'curqa:int,blmag:float,grmag:float,remag:float,nimag:float,s1mag:float,s2mag:float,'
        'thmag:float,blrmse:float,grrmse:float,rermse:float,nirmse:float,s1rmse:float,'
        's2rmse:float,thrmse:float,blcoef:array<float>,grcoef:array<float>,recoef:array<float>,'
        'nicoef:array<float>,s1coef:array<float>,s2coef:array<float>,thcoef:array<float>,'
        'blint:float,grint:float,reint:float,niint:float,s1int:float,s2int:float,thint:float,'
        'rfrawp:array<float>>')


def test_pixel_chip_schema():
    assert pixel.table() == 'pixel' and chip.table() == 'chip'
    assert pixel.schema().simpleString() == 'struct<cx:int,cy:int,px:int,py:int,mask:array<tinyint>>'
    assert chip.schema().simpleString() == 'struct<cx:int,cy:int,dates:array<string>>'


def test_timeseries_schema_names():
    assert timeseries.schema('ard').names == ['cx', 'cy', 'px', 'py', 'dates', 'blues', 'greens', 'reds',
                                             'nirs', 'swir1s', 'swir2s', 'thermals', 'qas']
    assert set(timeseries.schema('aux').names) == set(SCHEMABASE + ['aspect', 'dem', 'mpw', 'posidex', 'slope', 'trends'])
    assert set(timeseries.schema(None).keys()) == {'ard', 'aux'}


def test_segment_rows_projection():
    row = {k: i for i, k in enumerate(CCD_SCHEMA_NAMES)}
    row['extra'] = True
    proj = segment.rows([row])[0]
    assert list(proj.keys()) == segment.schema().fieldNames()


def test_format_snow_break_day_zero_raises_like_reference():
    """pyccd's permanent-snow / insufficient-clear models carry break_day = 0, and the
    reference's format calls date.fromordinal(0) (pyccd.py:115), which raises."""
    cm = {'start_day': 700000, 'end_day': 700100, 'break_day': 0}
    with pytest.raises(ValueError):
        pyccd.format(1, 2, 3, 4, [700000], {'change_models': [cm], 'processing_mask': [1]})


def test_pack_unpack_roundtrip():
    keys = timeseries.chip_keys(-1815585, 1064805, n_pix=6, width=3)
    assert keys[4] == (-1815585, 1064805, -1815585 + 30, 1064805 - 30)
    rng = np.random.default_rng(3)
    dates = np.array([734992, 734991, 734984], dtype=np.int64)
    spectra = rng.integers(-100, 5000, size=(7, 6, 3)).astype(np.int16)
    qa = rng.integers(0, 400, size=(6, 3)).astype(np.uint16)
    recs = timeseries.unpack(keys, dates, spectra, qa)
    k2, d2, s2, q2 = timeseries.pack(recs)
    assert k2 == keys and np.array_equal(d2, dates) and np.array_equal(s2, spectra) and np.array_equal(q2, qa)


def test_detect_partition_batches_and_matches_per_pixel(monkeypatch):
    """pyccd.rdd's partition function (mapPartitions) produces exactly the rows of per-record
    pyccd.detect; ccd's batched backend is answered here by the numpy restatement."""
    import ccd
    from ccdgpu import synth

    def fake_groups(groups, params=None):
        return [[ccd_ref.detect(dates, *[spectra[b, i] for b in range(7)], qas[i], params=params)
                 for i in range(qas.shape[0])] for dates, spectra, qas in groups]

    monkeypatch.setattr(ccd, 'detect_groups', fake_groups)
    monkeypatch.setattr(ccd, 'detect', ccd_ref.detect)
    d, s, q = synth.chip(synth.config(2), 9, 0, 3)
    d3, s3, q3 = synth.chip(synth.config(3), 1, 0, 2)  # a sidelap chip: another date vector
    recs = (timeseries.unpack(timeseries.chip_keys(0, 0, 3), d, s, q) + [TIMESERIES_ELEMENT] +
            timeseries.unpack(timeseries.chip_keys(3000, 0, 2), d3, s3, q3))
    rows = pyccd.detect_partition(recs)
    expected = [row for rec in recs for row in pyccd.detect(rec)]
    assert len(rows) == len(expected)
    for a, b in zip(rows, expected):
        assert a.keys() == b.keys()
        for k in a:
            if isinstance(a[k], float):
                assert a[k] == pytest.approx(b[k], rel=1e-12, nan_ok=True)
            else:
                assert a[k] == b[k]
