"""Transport-encoded uploads on the GPU (ccdgpu_stage_slot_encoded + ccd_decode_enc): the device
decode of an encoded batch equals the raw upload bit for bit -- encoded and raw-fallback chips,
both cadences, masked QA -- and detection of it returns the same segments."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def chips():
    from ccdgpu import synth
    out = [synth.chip(synth.config(3), 0, 0, 200), synth.chip(synth.config(3), 1, 0, 150),
           synth.chip(synth.config(4), 2, 0, 120)]
    # a chip with more than 16 distinct QA words (raw), from a C2 chip with shuffled clear words
    d, s, q = synth.chip(synth.config(2), 3, 0, 90)
    q = q.copy()
    clear = (q & 1) == 0
    rng = np.random.default_rng(9)
    q[clear] = np.where(rng.random(int(clear.sum())) < 0.5, q[clear], q[clear] | (rng.integers(0, 8, int(clear.sum())) << 11).astype(np.uint16))
    out.append((d, s, q))
    # a fill observation with data in a band (raw)
    d, s, q = synth.chip(synth.config(3), 4, 0, 60)
    s = s.copy()
    fi = np.argwhere((q & 1) == 1)[0]
    s[2, fi[0], fi[1]] = 123
    out.append((d, s, q))
    return out


def test_encoded_upload_decodes_to_the_raw_inputs_and_detects_the_same():
    import ccdgpu
    cs = chips()
    raw = ccdgpu.ChipBatch.from_chips(cs, pinned=True)
    enc = ccdgpu.EncodedBatch.encode(cs, threads=4)
    assert enc.chip_modes() == [1, 1, 1, 0, 0]
    assert enc.nbytes_encoded < raw.spectra.nbytes + raw.qa.nbytes
    ctx = ccdgpu.Context(0)
    try:
        ctx.stage_slot_chips(0, raw)
        ctx.run_slot(0)
        s0, q0 = ctx.staged_inputs()
        r0 = [ctx.fetch(c) for c in range(len(cs))]
        ctx.stage_slot_encoded(1, enc)
        ctx.run_slot(1)
        s1, q1 = ctx.staged_inputs()
        r1 = [ctx.fetch(c) for c in range(len(cs))]
    finally:
        ctx.close()
    np.testing.assert_array_equal(s1, np.asarray(raw.spectra))
    np.testing.assert_array_equal(q1, np.asarray(raw.qa))
    np.testing.assert_array_equal(s0, s1)
    np.testing.assert_array_equal(q0, q1)
    for a, b in zip(r0, r1):
        assert a.segments.tobytes() == b.segments.tobytes()
        assert np.array_equal(a.procedure, b.procedure) and np.array_equal(a.mask, b.mask)


def test_unread_drop_encoding_detects_the_same():
    """The runner's default encoding drops the band values of fill / cloud / shadow observations
    (never read by any procedure): the device gets -9999 there and the raw values elsewhere, and
    the detection -- segments, procedures, masks -- is the same as from the raw upload."""
    import ccdgpu
    from ccdgpu import synth
    cs = [synth.chip(synth.config(3), 5, 0, 300), synth.chip(synth.config(5), 6, 0, 200),
          synth.chip(synth.config(4), 7, 0, 200), synth.chip(synth.config(2), 8, 0, 150)]
    drop, strict = ccdgpu.unread_drop_bits(None)
    raw = ccdgpu.ChipBatch.from_chips(cs, pinned=True)
    enc = ccdgpu.EncodedBatch.encode(cs, threads=4, drop_bits=drop, strict_bits=strict)
    assert enc.nbytes_encoded < 0.65 * (raw.spectra.nbytes + raw.qa.nbytes)
    ctx = ccdgpu.Context(0)
    try:
        ctx.stage_slot_chips(0, raw)
        ctx.run_slot(0)
        r0 = [ctx.fetch(c) for c in range(len(cs))]
        ctx.stage_slot_encoded(1, enc)
        ctx.run_slot(1)
        s1, q1 = ctx.staged_inputs()
        r1 = [ctx.fetch(c) for c in range(len(cs))]
    finally:
        ctx.close()
    np.testing.assert_array_equal(q1, np.asarray(raw.qa))
    gone = (np.asarray(raw.qa) & drop) != 0
    s_raw = np.asarray(raw.spectra).reshape(-1)
    for c in range(len(cs)):
        d0, d1 = int(raw.data_off[c]), int(raw.data_off[c + 1])
        sr = s_raw[7 * d0:7 * d1].reshape(7, -1)
        se = s1[7 * d0:7 * d1].reshape(7, -1)
        g = gone[d0:d1]
        np.testing.assert_array_equal(se[:, ~g], sr[:, ~g])
        assert (se[:, g] == -9999).all()
    for a, b in zip(r0, r1):
        assert a.segments.tobytes() == b.segments.tobytes()
        assert np.array_equal(a.procedure, b.procedure) and np.array_equal(a.mask, b.mask)


def _corrupt(enc, fn):
    """a copy of an EncodedBatch with fn(buf, section offsets) applied to its bytes"""
    import copy
    b = copy.copy(enc)
    b.buf = enc.buf.copy()
    off = b.buf[8:8 * (b.n_chips + 2)].view(np.int64)
    fn(b.buf, [int(o) for o in off])
    return b


def test_malformed_encoded_batches_are_rejected():
    """ccdgpu_stage_slot_encoded checks every section against its mode's layout before the
    decoder reads it: a band stride below the kept count, a kept-offset table that does not end
    at kept or is not monotone, and a section too short for its columns are CCDGPU_EINVAL."""
    import ccdgpu
    from ccdgpu import synth
    cs = [synth.chip(synth.config(3), 0, 0, 64), synth.chip(synth.config(3), 1, 0, 40)]
    enc = ccdgpu.EncodedBatch.encode(cs, threads=2)
    assert enc.chip_modes() == [1, 1]

    def stride(buf, off):
        buf[off[0] + 64:off[0] + 72].view(np.int64)[0] = buf[off[0] + 48:off[0] + 56].view(np.int64)[0] - 8

    def stride_odd(buf, off):
        buf[off[0] + 64:off[0] + 72].view(np.int64)[0] += 4

    def koff_end(buf, off):
        buf[off[1] + 128 + 4 * 40:off[1] + 128 + 4 * 41].view(np.uint32)[0] -= 1

    def koff_order(buf, off):
        k = buf[off[0] + 128:off[0] + 128 + 4 * 65].view(np.uint32)
        k[3], k[4] = k[4] + 1, k[3]

    def huge_kept(buf, off):
        h = buf[off[0] + 48:off[0] + 72].view(np.int64)
        h[0] = h[2] = 64 * 1421 * 2

    ctx = ccdgpu.Context(0)
    try:
        for fn in (stride, stride_odd, koff_end, koff_order, huge_kept):
            with pytest.raises(ccdgpu.CcdGpuError) as ei:
                ctx.stage_slot_encoded(0, _corrupt(enc, fn))
            assert 'encoded batch' in str(ei.value), fn.__name__
        # the intact batch still stages and detects
        ctx.stage_slot_encoded(0, enc)
        ctx.run_slot(0)
    finally:
        ctx.close()


def test_restaging_the_slot_of_a_running_detection_is_rejected():
    """Between ccdgpu_run_slot_begin and _end only the other slot may be staged: staging the slot
    the running detection reads is CCDGPU_EINVAL (it would overwrite its inputs)."""
    import ccdgpu
    from ccdgpu import synth
    cs = [synth.chip(synth.config(3), 2, 0, 100)]
    raw = ccdgpu.ChipBatch.from_chips(cs, pinned=True)
    enc = ccdgpu.EncodedBatch.encode(cs, threads=2)
    ctx = ccdgpu.Context(0)
    try:
        ctx.stage_slot_chips(0, raw)
        ctx.run_slot_begin(0)
        for b in (raw, enc):
            with pytest.raises(ccdgpu.CcdGpuError) as ei:
                ctx.stage_slot_chips(0, b)
            assert 'run_slot_begin' in str(ei.value)
        ctx.stage_slot_chips(1, enc)  # the other slot is fine
        ctx.run_slot_end()
        r0 = ctx.fetch(0)
        ctx.run_slot(1)
        r1 = ctx.fetch(0)
    finally:
        ctx.close()
    assert r0.segments.tobytes() == r1.segments.tobytes()
