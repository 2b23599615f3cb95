"""The synthetic ARD generator is deterministic and subset-stable (bench and parity inputs)."""
import numpy as np

from ccdgpu import synth


def test_dates_descending_and_cadence():
    for which, lo, hi in ((2, 1000, 1000), (3, 1300, 2300), (5, 1300, 2300)):
        d = synth.dates(synth.config(which), 0)
        assert lo <= d.shape[0] <= hi
        assert np.all(np.diff(d) < 0)
        assert d.min() >= 723868 and d.max() <= 736694


def test_subset_regeneration_is_bit_identical():
    cfg = synth.config(5)
    d, s, q = synth.chip(cfg, 7, 0, 40)
    _, s2, q2 = synth.chip(cfg, 7, 25, 10, chip_dates=d)
    assert np.array_equal(s[:, 25:35], s2) and np.array_equal(q[25:35], q2)


def test_class_mix():
    d, s, q = synth.chip(synth.config(4), 2, 0, 50)
    fill = np.mean(q == 1)
    assert 0.05 < fill < 0.3
    assert np.all(s[:, q == 1] == -9999)
