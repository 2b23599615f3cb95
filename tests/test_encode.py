"""Transport encoding of chips for the PCIe upload (ccdgpu_encode_chips, include/ccdgpu.h): the
encoded bytes decode -- with a numpy restatement of the device decoder (ccd_decode_enc,
ccd_pack.hip) -- to the original spectra and QA bit for bit, for encoded and raw-fallback chips,
and the AVX-512 VBMI2 and scalar encoders write the same bytes.  CPU only (no device)."""
import os
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, 'lcmap-firebird_amd'))

ccdgpu = pytest.importorskip('ccdgpu')
from ccdgpu import synth  # noqa: E402


from encode_util import decode  # noqa: E402


def encode(chips, threads=3, drop=1, strict=1):
    e = ccdgpu.EncodedBatch.encode(chips, threads=threads, pinned=False, drop_bits=drop, strict_bits=strict)
    return e, e.buf[:e.nbytes_encoded]


def check_roundtrip(chips, modes=None):
    e, buf = encode(chips)
    dec = decode(buf)
    for (d, s, q), (ds, dq) in zip(chips, dec):
        np.testing.assert_array_equal(ds, s)
        np.testing.assert_array_equal(dq, q)
    if modes is not None:
        assert e.chip_modes() == modes
    return e


def test_synthetic_tile_chips_roundtrip_and_shrink():
    cfg = synth.config(3)
    chips = [synth.chip(cfg, c, 0, 300) for c in (0, 1, 2)]  # base cadence and sidelap
    e = check_roundtrip(chips, [1, 1, 1])
    raw = sum(s.nbytes + q.nbytes for _, s, q in chips)
    assert e.nbytes_encoded < 0.9 * raw


def test_masked_and_change_dense_configs_roundtrip():
    for which in (2, 4, 5):
        cfg = synth.config(which)
        check_roundtrip([synth.chip(cfg, 7, 0, 128), synth.chip(cfg, 8, 0, 77)])


def test_raw_fallbacks_and_edge_shapes():
    rng = np.random.default_rng(5)
    n = 33  # odd observation count: the last QA byte holds one code
    d = np.arange(n, dtype=np.int64) * 16 + 730000
    # more than 16 distinct QA words -> raw
    q_many = rng.integers(2, 4000, size=(5, n)).astype(np.uint16) & ~np.uint16(1)
    s_many = rng.integers(-100, 10000, size=(7, 5, n)).astype(np.int16)
    # a fill observation (QA bit 0) whose bands are not all -9999 -> raw
    q_bad = np.full((3, n), 66, dtype=np.uint16)
    q_bad[1, 4] = 1
    s_bad = rng.integers(0, 5000, size=(7, 3, n)).astype(np.int16)
    s_bad[:, 1, 4] = -9999
    s_bad[3, 1, 4] = 17
    # all observations fill (nothing kept), one pixel
    q_fill = np.ones((1, n), dtype=np.uint16)
    s_fill = np.full((7, 1, n), -9999, dtype=np.int16)
    # a single observation
    q_one = np.array([[322]], dtype=np.uint16)
    s_one = np.array([[[5]], [[6]], [[7]], [[8]], [[9]], [[10]], [[11]]], dtype=np.int16)
    check_roundtrip([(d, s_many, q_many), (d, s_bad, q_bad), (d, s_fill, q_fill), (d[:1], s_one, q_one)],
                    [0, 0, 1, 1])


def test_vector_and_scalar_encoders_write_the_same_bytes():
    code = ("import sys, numpy as np; sys.path.insert(0, %r); import ccdgpu; from ccdgpu import synth; "
            "cfg = synth.config(3); chips = [synth.chip(cfg, c, 0, 97) for c in (0, 1)]; "
            "e = ccdgpu.EncodedBatch.encode(chips, threads=2, pinned=False); "
            "sys.stdout.buffer.write(bytes([int(ccdgpu.encode_vector_path())]) + e.buf[:e.nbytes_encoded].tobytes())"
            % os.path.join(ROOT, 'lcmap-firebird_amd'))
    outs = {}
    for scalar in ('0', '1'):
        env = dict(os.environ, CCDGPU_ENCODE_SCALAR=scalar)
        outs[scalar] = subprocess.run([sys.executable, '-c', code], env=env, capture_output=True, check=True).stdout
    assert outs['1'][0] == 0
    if outs['0'][0] == 0:
        pytest.skip('no AVX-512 VBMI2 on this CPU: only the scalar encoder ran')
    assert outs['0'][1:] == outs['1'][1:]


def test_unread_observations_dropped_and_the_rest_kept():
    """drop = fill | cloud | shadow bits: the observations of those classes come back as -9999,
    every other one (clear, water, snow, any other word) bit for bit; QA words all kept."""
    drop, strict = ccdgpu.unread_drop_bits(None)
    assert (drop, strict) == ((1 << 0) | (1 << 5) | (1 << 3), 1)
    cfg = synth.config(3)
    chips = [synth.chip(cfg, c, 0, 200) for c in (0, 1)]
    e, buf = encode(chips, drop=drop, strict=strict)
    raw = sum(s.nbytes + q.nbytes for _, s, q in chips)
    assert e.nbytes_encoded < 0.6 * raw
    for (d, s, q), (ds, dq) in zip(chips, decode(buf)):
        np.testing.assert_array_equal(dq, q)
        gone = (q & drop) != 0
        np.testing.assert_array_equal(ds[:, ~gone], s[:, ~gone])
        assert (ds[:, gone] == -9999).all()


def test_encode_rejects_a_short_buffer():
    cfg = synth.config(3)
    d, s, q = synth.chip(cfg, 0, 0, 10)
    e = ccdgpu.EncodedBatch([10], [d.shape[0]], pinned=False)
    e.buf = e.buf[:100]
    with pytest.raises(ValueError):
        e.fill([(d, s, q)])


def test_word_outside_the_palette_sample_reencodes_the_same_bytes():
    """The vector encoder takes the palette from every 16th pixel's QA row and re-encodes a chip
    whose other rows hold a word the sample missed: the result decodes to the inputs and matches
    the scalar encoder (which scans every row) byte for byte."""
    code = ("import sys, numpy as np; sys.path.insert(0, %r); import ccdgpu; "
            "n = 45; rng = np.random.default_rng(3); d = np.arange(n, dtype=np.int64) * 16 + 730000; "
            "q = np.full((40, n), 322, dtype=np.uint16); q[5, 3] = 324; q[17, 0] = 480; q[39, n - 1] = 1; "
            "s = rng.integers(0, 5000, size=(7, 40, n)).astype(np.int16); s[:, 39, n - 1] = -9999; "
            "e = ccdgpu.EncodedBatch.encode([(d, s, q)], threads=2, pinned=False); "
            "sys.stdout.buffer.write(bytes([int(ccdgpu.encode_vector_path())]) + e.buf[:e.nbytes_encoded].tobytes())"
            % os.path.join(ROOT, 'lcmap-firebird_amd'))
    outs = {}
    for scalar in ('0', '1'):
        env = dict(os.environ, CCDGPU_ENCODE_SCALAR=scalar)
        outs[scalar] = subprocess.run([sys.executable, '-c', code], env=env, capture_output=True, check=True).stdout
    buf = np.frombuffer(outs['0'][1:], dtype=np.uint8)
    rng = np.random.default_rng(3)
    n = 45
    q = np.full((40, n), 322, dtype=np.uint16)
    q[5, 3] = 324
    q[17, 0] = 480
    q[39, n - 1] = 1
    s = rng.integers(0, 5000, size=(7, 40, n)).astype(np.int16)
    s[:, 39, n - 1] = -9999
    (ds, dq), = decode(buf)
    np.testing.assert_array_equal(ds, s)
    np.testing.assert_array_equal(dq, q)
    if outs['0'][0] == 0:
        pytest.skip('no AVX-512 VBMI2 on this CPU: only the scalar encoder ran')
    assert outs['0'][1:] == outs['1'][1:]


def test_scalar_encoder_dropped_last_observation_at_thread_boundaries():
    """Scalar encoder (CCDGPU_ENCODE_SCALAR=1), 4 threads, the 'unread' drop: every pixel's last
    observation is a dropped (cloud) one with data in its bands, and the kept total is a multiple
    of 8 (band stride = kept total, no padding).  The scalar compaction once wrote each dropped
    value one past the pixel's kept run -- over the next pixel's first kept value (the next
    thread's, at a chunk boundary) or, after the last pixel, over the next band's first value."""
    code = ("import sys, numpy as np; sys.path.insert(0, %r); import ccdgpu; "
            "n = 21; P = 64; rng = np.random.default_rng(11); d = np.arange(n, dtype=np.int64) * 16 + 730000; "
            "q = np.full((P, n), 322, dtype=np.uint16); q[:, n - 1] = 322 | 32; q[:, 4] = 1; "
            "s = rng.integers(0, 5000, size=(7, P, n)).astype(np.int16); s[:, :, 4] = -9999; "
            "drop, strict = ccdgpu.unread_drop_bits(None); "
            "e = ccdgpu.EncodedBatch.encode([(d, s, q)], threads=4, pinned=False, drop_bits=drop, strict_bits=strict); "
            "sys.stdout.buffer.write(e.buf[:e.nbytes_encoded].tobytes())"
            % os.path.join(ROOT, 'lcmap-firebird_amd'))
    env = dict(os.environ, CCDGPU_ENCODE_SCALAR='1')
    out = subprocess.run([sys.executable, '-c', code], env=env, capture_output=True, check=True).stdout
    n, P = 21, 64
    assert (P * (n - 2)) % 8 == 0
    rng = np.random.default_rng(11)
    q = np.full((P, n), 322, dtype=np.uint16)
    q[:, n - 1] = 322 | 32
    q[:, 4] = 1
    s = rng.integers(0, 5000, size=(7, P, n)).astype(np.int16)
    s[:, :, 4] = -9999
    (ds, dq), = decode(np.frombuffer(out, dtype=np.uint8))
    np.testing.assert_array_equal(dq, q)
    keep = np.ones(n, dtype=bool)
    keep[[4, n - 1]] = False
    np.testing.assert_array_equal(ds[:, :, keep], s[:, :, keep])
    assert (ds[:, :, ~keep] == -9999).all()


def test_encoded_check_rejects_malformed_batches_on_the_host():
    """ccdgpu_encoded_check (the checks ccdgpu_stage_slot_encoded makes before the upload; no
    device): a band stride below the kept count or not a multiple of 8, a kept-offset table that
    does not end at kept or is not monotone, a kept count past the chip, a truncated section and a
    shape mismatch are rejected; the intact batch passes."""
    cs = [synth.chip(synth.config(3), 0, 0, 64), synth.chip(synth.config(3), 1, 0, 40)]
    e, _ = encode(cs, threads=2)
    assert e.chip_modes() == [1, 1]
    e.check()
    off = [int(o) for o in e.buf[8:8 * (e.n_chips + 2)].view(np.int64)]

    def corrupt(fn):
        import copy
        b = copy.copy(e)
        b.buf = e.buf.copy()
        fn(b)
        with pytest.raises(ccdgpu.CcdGpuError, match='encoded batch'):
            b.check()

    def h64(b, k):
        return b.buf[off[k] + 48:off[k] + 80].view(np.int64)

    def koff(b, k, n):
        return b.buf[off[k] + 128:off[k] + 128 + 4 * (n + 1)].view(np.uint32)

    corrupt(lambda b: h64(b, 0).__setitem__(2, h64(b, 0)[0] - 8))
    corrupt(lambda b: h64(b, 0).__setitem__(2, h64(b, 0)[2] + 4))
    corrupt(lambda b: koff(b, 1, 40).__setitem__(40, koff(b, 1, 40)[40] - 1))
    corrupt(lambda b: koff(b, 0, 64).__setitem__(slice(3, 5), [koff(b, 0, 64)[4] + 1, koff(b, 0, 64)[3]]))
    corrupt(lambda b: h64(b, 0).__setitem__(slice(0, 3, 2), [64 * 1421 * 2, 64 * 1421 * 2]))
    corrupt(lambda b: setattr(b, 'nbytes_encoded', off[2] - 64))
    corrupt(lambda b: b.buf[off[1] + 4:off[1] + 8].view(np.int32).__setitem__(0, 41))


@pytest.mark.parametrize('nt', ['1', '0'])
def test_streaming_writer_fills_exactly_its_range(tmp_path, nt):
    """The encoder's streaming writer (ntw_*: band runs staged in L1, full lines out with
    non-temporal stores, the ranges' shared first / last lines with masked ordinary stores) on
    400 random ranges -- any start alignment, 0..32 values per append -- writes every value of its
    range and nothing outside it (tests/native/ntw_check.c; AVX-512F/BW, no VBMI2 needed)."""
    exe = str(tmp_path / 'ntw_check')
    subprocess.run(['gcc', '-O2', '-fopenmp', '-I', os.path.join(ROOT, 'include'), '-o', exe,
                    os.path.join(HERE, 'native', 'ntw_check.c')], check=True)
    out = subprocess.run([exe], env=dict(os.environ, CCDGPU_ENCODE_NT=nt), capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    if out.stdout.startswith('skip'):
        pytest.skip(out.stdout.strip())
    assert out.stdout.strip() == 'ok'
