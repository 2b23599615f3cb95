"""The device generator (ccdsynth_gpu_*, csrc/ccd_synth.hip) against the host generator
(ccdsynth_chip): both run the arithmetic of csrc/synth_core.h, so whole chips must agree to the
bit (the math libraries' cos / log may differ by an ulp, which could move an int16 sample only
within ~1e-12 of a half-integer: none in these chips).  The tile-parity run and the bench's tile
leg use the device generator for the tile's 2500 distinct chips."""
import numpy as np
import pytest

from ccdgpu import synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('which,chips,n_pix', [(3, [0, 1, 2], 600), (5, [3, 2498], 400), (4, [11], 300), (2, [5], 300)])
def test_device_generator_equals_host_generator(which, chips, n_pix):
    cfg = synth.config(which)
    g = synth.DeviceGenerator(0)
    b = g.batch(cfg, chips, n_pix=n_pix, pix0=123)
    g.close()
    for j, c in enumerate(chips):
        d, s, q = synth.chip(cfg, c, 123, n_pix)
        bd, bs, bq = b.chip(j)
        assert np.array_equal(bd, d)
        assert np.array_equal(bq, q), (c, int(np.count_nonzero(bq != q)))
        assert np.array_equal(bs, s), (c, int(np.count_nonzero(bs != s)))


def test_device_generator_reuses_its_output_batch():
    cfg = synth.config(3)
    g = synth.DeviceGenerator(0)
    b = g.batch(cfg, [7, 9], n_pix=200)
    first = (b.spectra.copy(), b.qa.copy())
    b2 = g.batch(cfg, [7, 9], n_pix=200, out=b)
    assert b2 is b and np.array_equal(first[0], b.spectra) and np.array_equal(first[1], b.qa)
    with pytest.raises(ValueError):
        g.batch(cfg, [7, 10], n_pix=200, out=b) if synth.dates(cfg, 10).shape != synth.dates(cfg, 9).shape \
            else g.batch(cfg, [7, 9], n_pix=100, out=b)
    g.close()
