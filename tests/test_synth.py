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


class _HostGen(object):
    """DeviceGenerator stand-in on the host (same samples: synth_core.h)."""

    def batch(self, cfg, ids, n_pix=10000, pix0=0, out=None, pinned=False):
        import ccdgpu
        if out is None:
            out = ccdgpu.ChipBatch([n_pix] * len(ids), [synth.dates(cfg, c).shape[0] for c in ids])
        for j, c in enumerate(ids):
            synth.chip(cfg, c, pix0, n_pix, out=out.chip(j))
        return out

    def dates(self, cfg, c):
        return synth.dates(cfg, c)

    def close(self):
        pass


def test_tile_source_pool_mode_serves_distinct_chips(monkeypatch):
    """TileSource 'pool' mode (the bench's tile leg): every position gets a copy of a pool chip of
    its own cadence with its dates moved by a multiple of 16 days; positions differ; buffers
    recycle."""
    import numpy as np
    monkeypatch.setattr(synth.TileSource, '_gen', lambda self: _HostGen())
    cfg = synth.config(3)
    src = synth.TileSource(cfg, batch_chips=4, n_pix=12, mode='pool', pool_chips=6, pinned=False, rotate_threads=2)
    src.prepare()
    seen = set()
    for pos0 in (0, 4, 8):
        pos = list(range(pos0, pos0 + 4))
        b = src(pos)
        for j, p in enumerate(pos):
            d, s, q = b.chip(j)
            d0 = synth.dates(cfg, p)
            (cid, pd, ps, pq), days = src._pool_chip(p, p, d0)
            assert days % 16 == 0 and 16 <= days <= 1024
            assert np.array_equal(d, d0 + days) and np.array_equal(pd, d0)
            assert np.array_equal(s, ps) and np.array_equal(q, pq)
            seen.add((cid, d.tobytes()))
        src.release(b)
    assert len(seen) == 12  # every position distinct
    assert src.allocated == 1  # the released buffer was reused
