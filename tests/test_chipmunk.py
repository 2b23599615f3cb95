"""Chip packer: chipmunk wire format -> detection layout.  CPU tests pin
the host side (ubid map against the reference's registry fixture, grouping, text layout) and
the numpy restatement against the reference's chip fixture; GPU tests check the device decode +
pivot bit-exactly against it and the end-to-end detection from chips."""
import json
import os

import numpy as np
import pytest

import chipmunk_ref
from ccdc import chipmunk

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'chipmunk')


def load(name):
    with open(os.path.join(FIX, name)) as f:
        return json.load(f)


def synthetic(n_pix=97, n_obs=37, seed=3, x=-1815585, y=1064805):
    rng = np.random.default_rng(seed)
    dates = np.sort(rng.choice(np.arange(724000, 736500), n_obs, replace=False))[::-1].astype(np.int64)
    spectra = rng.integers(-32768, 32767, size=(7, n_pix, n_obs), dtype=np.int16)
    qa = rng.integers(0, 65535, size=(n_pix, n_obs), dtype=np.uint16)
    return dates, spectra, qa, chipmunk.chip_response(x, y, dates, spectra, qa)


def test_ubid_map_matches_reference_registry():
    assert chipmunk.check_registry(load('registry_response.json'))


def test_registry_check_rejects_a_wrong_map(monkeypatch):
    bad = dict(chipmunk.ARD_UBIDS, blues=('LC08_SRB3',) + chipmunk.ARD_UBIDS['blues'][1:])
    monkeypatch.setattr(chipmunk, 'ARD_UBIDS', bad)
    with pytest.raises(ValueError):
        chipmunk.check_registry(load('registry_response.json'))


def test_reference_chip_fixture():
    """test/data/chip_response.json: one le07_srb1 chip of (-1815585, 1064805) on 2002-12-21,
    all fill.  It is a blue layer; alone it is asymmetric (merlin would reject it)."""
    chips = load('chip_response.json')
    g = chipmunk.group(chips)
    assert list(g) == [(-1815585, 1064805)]
    layers = g[(-1815585, 1064805)]
    d = chipmunk.ordinal('2002-12-21T00:00:00Z')
    assert list(layers['blues']) == [d] and all(not layers[n] for n in chipmunk.LAYERS[1:])
    with pytest.raises(ValueError):
        chipmunk.dates_of(layers)
    dates, text, offsets = chipmunk.pack_text([layers], symmetric=False)
    assert dates.tolist() == [[d]] and offsets[0, 0].tolist() == [0, -1, -1, -1, -1, -1, -1, -1]
    n_pix = chipmunk.payload_pixels(chips[0]['data'])
    assert n_pix == 10000
    spectra, qa = chipmunk_ref.decode(dates, text, offsets, n_pix)
    assert (spectra == -9999).all() and (qa == 1).all()


def test_group_and_text_round_trip():
    dates, spectra, qa, chips = synthetic()
    rng = np.random.default_rng(0)
    chips = [chips[i] for i in rng.permutation(len(chips))]  # chipmunk order is arbitrary
    g = chipmunk.group(chips)
    (key, layers), = g.items()
    d, text, offsets = chipmunk.pack_text([layers])
    assert np.array_equal(d[0], dates)  # descending, as merlin delivers
    s2, q2 = chipmunk_ref.decode(d, text, offsets, spectra.shape[1])
    assert np.array_equal(s2[0], spectra) and np.array_equal(q2[0], qa)


def test_duplicate_layer_rejected():
    _, _, _, chips = synthetic(n_pix=4, n_obs=2)
    with pytest.raises(ValueError):
        chipmunk.group(chips + chips[:1])


@pytest.mark.gpu
def test_device_unpack_matches_host_restatement():
    import ccdgpu
    ctx = ccdgpu.Context(0)
    locs, refs = [], []
    for seed, (x, y) in enumerate([(0, 0), (3000, 0), (0, -3000)]):
        dates, spectra, qa, chips = synthetic(n_pix=10000, n_obs=150, seed=11)  # shared dates
        spectra = np.roll(spectra, seed, axis=1)
        qa = np.roll(qa, seed, axis=0)
        chips = chipmunk.chip_response(x, y, dates, spectra, qa)
        locs.append(chipmunk.group(chips)[(x, y)])
        refs.append((spectra, qa))
    d, text, offsets = chipmunk.pack_text(locs)
    offsets[1, 5, 3] = -1  # one missing layer -> fill
    secs = ctx.stage_chipmunk(d, text, offsets, 10000)
    assert secs > 0
    es, eq = chipmunk_ref.decode(d, text, offsets, 10000)
    got_s, got_q = ctx.staged_inputs()
    assert np.array_equal(got_s, es) and np.array_equal(got_q, eq)
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize('n_pix,n_obs', [(97, 131), (98, 129), (10000, 257)])
def test_device_unpack_unaligned_payloads(n_pix, n_obs):
    """Payloads at every offset mod 4 (the kernel's 8-character loads are then unaligned), with
    '#' between them (never decoded), '=' and '==' padding (97 / 98 pixels) and partial tiles
    of both dimensions."""
    import ccdgpu
    ctx = ccdgpu.Context(0)
    dates, spectra, qa, chips = synthetic(n_pix=n_pix, n_obs=n_obs, seed=5)
    d, text, offsets = chipmunk.pack_text([chipmunk.group(chips)[(-1815585, 1064805)]])
    enc = 4 * ((2 * n_pix + 2) // 3)
    out, shifted = bytearray(), np.full_like(offsets, -1)
    for i, (o, l) in enumerate(np.ndindex(*offsets.shape[1:])):
        if offsets[0, o, l] < 0:
            continue
        out += b'#' * (i % 4)
        shifted[0, o, l] = len(out)
        out += text[offsets[0, o, l]:offsets[0, o, l] + enc]
    shifted[0, 3, 1] = -1
    ctx.stage_chipmunk(d, bytes(out), shifted, n_pix)
    es, eq = chipmunk_ref.decode(d, bytes(out), shifted, n_pix)
    got_s, got_q = ctx.staged_inputs()
    assert np.array_equal(got_s, es) and np.array_equal(got_q, eq)
    ctx.close()


@pytest.mark.gpu
def test_device_unpack_rejects_bad_base64():
    import ccdgpu
    ctx = ccdgpu.Context(0)
    dates, spectra, qa, chips = synthetic(n_pix=50, n_obs=4)
    d, text, offsets = chipmunk.pack_text([chipmunk.group(chips)[(-1815585, 1064805)]])
    bad = bytearray(text)
    bad[offsets[0, 2, 4] + 5] = ord('!')
    with pytest.raises(ccdgpu.CcdGpuError):
        ctx.stage_chipmunk(d, bytes(bad), offsets, 50)
    with pytest.raises(ccdgpu.CcdGpuError):  # payload past the end of the text
        ctx.stage_chipmunk(d, text[:-10], offsets, 50)
    pad = bytearray(text)
    pad[offsets[0, 1, 7] + 8] = ord('=')  # padding in the first place of a quantum
    with pytest.raises(ccdgpu.CcdGpuError):
        ctx.stage_chipmunk(d, bytes(pad), offsets, 50)
    ctx.stage_chipmunk(d, text, offsets, 50)  # the context still stages a good text afterwards
    ctx.close()


@pytest.mark.gpu
def test_detect_chips_equals_record_path():
    """Rows from chipmunk chips (device decode) == rows from merlin-style records (host arrays)."""
    from ccdc import pyccd, timeseries
    from ccdgpu import synth
    d, s, q = synth.chip(synth.config(2), 5, 0, 300)
    order = np.argsort(d)[::-1]  # merlin delivers dates descending
    d, s, q = d[order], s[:, :, order], q[:, order]
    x, y = -1815585, 1064805
    rows = pyccd.detect_chips(chipmunk.chip_response(x, y, d, s, q))
    records = timeseries.unpack(timeseries.chip_keys(x, y, 300), d, s, q)
    ref = pyccd.detect_partition(records)
    assert len(rows) == len(ref) > 300
    for a, b in zip(rows, ref):
        assert a == b


def test_sink_schemas_follow_reference():
    """Arrow schemas of the sink = the reference Spark schemas (names, order, storage types)."""
    import pyarrow as pa
    from ccdc import chip, pixel, pyccd, segment, sink
    for sch in (pyccd.schema(), segment.schema(), pixel.schema(), chip.schema()):
        a = sink.arrow_schema(sch)
        assert a.names == sch.fieldNames()
        for f, g in zip(sch, a):
            want = {'int': pa.int32(), 'float': pa.float32(), 'string': pa.string(),
                    'array<float>': pa.list_(pa.float32()), 'array<string>': pa.list_(pa.string()),
                    'array<tinyint>': pa.list_(pa.int8())}[f.dataType.simpleString()]
            assert g.type == want, f.name


def test_sink_tables_from_rows_and_default_row(tmp_path):
    from ccdc import sink
    from ccdgpu import abi
    rows = np.zeros(3, abi.ROW_DTYPE)
    rows['px'], rows['py'] = [30, 30, 60], [0, 0, 0]
    rows['sday'], rows['eday'], rows['bday'] = [723000, 724000, 1], [723500, 725000, 1], [723600, 725100, 1]
    rows['has_model'] = [1, 1, 0]
    rows['chprob'] = [1.0, 0.0, 0.0]
    rows['curqa'] = [8, 24, 0]
    rows['coef'][:2] = np.arange(49, dtype=np.float32).reshape(7, 7)
    off = np.array([0, 2, 3])
    mask = np.array([[1, 0, 1], [0, 0, 0]], dtype=np.int8)
    t = sink.tables(0, 0, np.array([723001, 723000, 723010]), off, rows, mask)
    seg = t['segment'].to_pylist()
    assert seg[0]['sday'] == '1980-07-04' == __import__('datetime').date.fromordinal(723000).isoformat()
    assert seg[2]['sday'] == seg[2]['bday'] == '0001-01-01' and seg[2]['blmag'] is None and seg[2]['curqa'] is None
    assert seg[0]['grcoef'] == [float(x) for x in range(7, 14)] and seg[2]['grcoef'] is None
    pix = t['pixel'].to_pylist()
    assert [(p['px'], p['mask']) for p in pix] == [(30, [1, 0, 1]), (60, [0, 0, 0])]
    assert t['chip'].to_pylist()[0]['dates'][0] == __import__('datetime').date.fromordinal(723001).isoformat()
    paths = sink.write_parquet(str(tmp_path), t, 0, 0)
    import pyarrow.parquet as pq
    assert pq.read_table(paths['segment']).equals(t['segment'])


@pytest.mark.gpu
def test_device_rows_equal_formatted_rows_cast_to_float32():
    """Output writer: device-packed rows == pyccd.format rows after Spark's float32 cast."""
    from ccdc import pyccd, sink
    from ccdgpu import synth
    d, s, q = synth.chip(synth.config(5), 2, 0, 200)
    order = np.argsort(d)[::-1]
    d, s, q = d[order], s[:, :, order], q[:, order]
    chips = chipmunk.chip_response(-1815585, 1064805, d, s, q)
    ref = pyccd.detect_chips(chips)
    (key, t), = pyccd.detect_chips_tables(chips)
    seg = t['segment'].to_pylist()
    assert len(seg) == len(ref) > 200
    f32 = lambda v: None if v is None else float(np.float32(v))
    for a, b in zip(seg, ref):
        for k in a:
            if k == 'rfrawp':
                assert a[k] is None
            elif k.endswith('coef'):
                assert a[k] == (None if b[k] is None else [f32(x) for x in b[k]]), k
            elif k in ('chprob',) or k.endswith('mag') or k.endswith('rmse') or k.endswith('int'):
                assert a[k] == f32(b[k]), k
            else:
                assert a[k] == b[k], k
    pix = t['pixel'].to_pylist()
    first_rows = {}
    for r in ref:
        first_rows.setdefault((r['px'], r['py']), r)
    assert len(pix) == 200
    for p in pix:
        assert p['mask'] == [int(x) for x in first_rows[(p['px'], p['py'])]['mask']]
    assert t['chip'].to_pylist()[0]['dates'] == ref[0]['dates']
