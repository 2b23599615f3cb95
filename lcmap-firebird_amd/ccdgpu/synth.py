"""ctypes binding for the synthetic ARD generator (lib/libccdsynth.so, include/ccdsynth.h).

Bench/test input only: stands in for merlin.create (reference ccdc/timeseries.py:120).
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(os.path.dirname(_HERE), 'lib', 'libccdsynth.so')


class SynthCfg(ctypes.Structure):
    _fields_ = [('n_obs_target', ctypes.c_int32), ('sidelap', ctypes.c_int32),
                ('change_every_days', ctypes.c_int32), ('first_year_l4', ctypes.c_int32),
                ('p_clear', ctypes.c_double), ('p_cloud', ctypes.c_double),
                ('p_shadow', ctypes.c_double), ('p_snow', ctypes.c_double),
                ('p_water', ctypes.c_double), ('p_fill', ctypes.c_double),
                ('p_saturated', ctypes.c_double), ('p_hot_thermal', ctypes.c_double),
                ('seed', ctypes.c_uint64)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise RuntimeError('libccdsynth.so not built: run __graft_entry__.build()')
        L = ctypes.CDLL(_LIB_PATH)
        L.ccdsynth_config.argtypes = [ctypes.c_int, ctypes.POINTER(SynthCfg)]
        L.ccdsynth_dates.argtypes = [ctypes.POINTER(SynthCfg), ctypes.c_int32,
                                     ctypes.c_void_p, ctypes.c_int32]
        L.ccdsynth_chip.argtypes = [ctypes.POINTER(SynthCfg), ctypes.c_int32, ctypes.c_int32,
                                    ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_void_p]
        L.ccdsynth_gpu_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        L.ccdsynth_gpu_destroy.argtypes = [ctypes.c_void_p]
        L.ccdsynth_gpu_error.restype = ctypes.c_char_p
        L.ccdsynth_gpu_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(SynthCfg), ctypes.c_int32] + [ctypes.c_void_p] * 9
        L.ccdsynth_rotate.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32]
        _lib = L
    return _lib


def config(which, **overrides):
    c = SynthCfg()
    if lib().ccdsynth_config(int(which), ctypes.byref(c)) != 0:
        raise ValueError('unknown synthetic config %r' % (which,))
    for k, v in overrides.items():
        setattr(c, k, v)
    return c


def dates(cfg, chip):
    n = lib().ccdsynth_dates(ctypes.byref(cfg), int(chip), None, 0)
    out = np.empty(n, dtype=np.int64)
    lib().ccdsynth_dates(ctypes.byref(cfg), int(chip), out.ctypes.data, n)
    return out


def chip(cfg, chip_index, pix0=0, n_pix=10000, chip_dates=None, out=None):
    """Returns (dates[n] descending int64, spectra[7][n_pix][n] int16, qa[n_pix][n] uint16).
    out=(dates, spectra, qa): C-contiguous arrays of those shapes to fill in place (e.g. the
    views of ccdgpu.ChipBatch.chip)."""
    d = dates(cfg, chip_index) if chip_dates is None else np.ascontiguousarray(chip_dates, dtype=np.int64)
    n = d.shape[0]
    if out is not None:
        od, spectra, qa = out
        if (od.shape != (n,) or spectra.shape != (7, n_pix, n) or qa.shape != (n_pix, n) or
                not (od.flags.c_contiguous and spectra.flags.c_contiguous and qa.flags.c_contiguous) or
                od.dtype != np.int64 or spectra.dtype != np.int16 or qa.dtype != np.uint16):
            raise ValueError('out arrays do not match chip %d (n_obs %d, n_pix %d)' % (chip_index, n, n_pix))
        od[...] = d
        d = od
    else:
        spectra = np.empty((7, n_pix, n), dtype=np.int16)
        qa = np.empty((n_pix, n), dtype=np.uint16)
    lib().ccdsynth_chip(ctypes.byref(cfg), int(chip_index), int(pix0), int(n_pix), int(n),
                        d.ctypes.data, spectra.ctypes.data, qa.ctypes.data)
    return d, spectra, qa


class DeviceGenerator(object):
    """The generator on a GPU (ccdsynth_gpu_*, csrc/ccd_synth.hip): the same samples as ``chip``
    for whole batches of chips, computed in HBM and copied into a ``ccdgpu.ChipBatch`` (pinned for
    full PCIe rate).  For inputs too large to generate on the host, e.g. a tile's 2500 distinct
    chips.  Not thread-safe: one generator per thread."""

    def __init__(self, device=0):
        self._g = ctypes.c_void_p()
        if lib().ccdsynth_gpu_create(int(device), ctypes.byref(self._g)) != 0:
            raise RuntimeError('ccdsynth_gpu_create: %s' % lib().ccdsynth_gpu_error().decode())
        self._dates = {}

    def close(self):
        if self._g:
            lib().ccdsynth_gpu_destroy(self._g)
            self._g = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def dates(self, cfg, c):
        key = (bytes(cfg), int(c))
        d = self._dates.get(key)
        if d is None:
            d = self._dates[key] = dates(cfg, c)
        return d

    def batch(self, cfg, chip_ids, n_pix=10000, pix0=0, out=None, pinned=True):
        """Chips ``chip_ids`` (pixels pix0 .. pix0+n_pix-1 of each) as a ChipBatch: ``out`` when
        given (its chip shapes must match), else a new one."""
        import ccdgpu
        ids = [int(c) for c in chip_ids]
        nobs = [self.dates(cfg, c).shape[0] for c in ids]
        if out is None:
            out = ccdgpu.ChipBatch([n_pix] * len(ids), nobs, pinned=pinned)
        elif list(out.n_obs) != nobs or list(out.n_pix) != [n_pix] * len(ids):
            raise ValueError('out batch does not match the chips %s' % (ids,))
        for j, c in enumerate(ids):
            out.dates[out.obs_off[j]:out.obs_off[j + 1]] = self.dates(cfg, c)
        a32 = lambda v: np.ascontiguousarray(v, dtype=np.int32)
        cid, p0, npx, nob = a32(ids), a32([pix0] * len(ids)), a32(out.n_pix), a32(out.n_obs)
        oo, do = np.ascontiguousarray(out.obs_off[:-1]), np.ascontiguousarray(out.data_off[:-1])
        rc = lib().ccdsynth_gpu_batch(self._g, ctypes.byref(cfg), len(ids), cid.ctypes.data, p0.ctypes.data,
                                      npx.ctypes.data, nob.ctypes.data, oo.ctypes.data, do.ctypes.data,
                                      out.dates.ctypes.data, out.spectra.ctypes.data, out.qa.ctypes.data)
        if rc != 0:
            raise RuntimeError('ccdsynth_gpu_batch: %s' % lib().ccdsynth_gpu_error().decode())
        return out


def rotate(spectra, qa, shift, out_spectra, out_qa, threads=8):
    """out = the chip with every pixel series rotated left by ``shift`` observations (same
    dates): out[..., i] = in[..., (i + shift) mod n] for the 7 bands and the QA (ccdsynth_rotate)."""
    n_pix, n = qa.shape
    assert spectra.shape == (7, n_pix, n) and out_spectra.shape == spectra.shape and out_qa.shape == qa.shape
    for a in (spectra, qa, out_spectra, out_qa):
        assert a.flags.c_contiguous
    if lib().ccdsynth_rotate(spectra.ctypes.data, qa.ctypes.data, n_pix, n, int(shift), out_spectra.ctypes.data,
                             out_qa.ctypes.data, int(threads)) != 0:
        raise ValueError('ccdsynth_rotate failed')


class TileSource(object):
    """``source(positions) -> ChipBatch`` for ccdc.runner: the tile chips at those positions, each
    one distinct, in pinned buffers from a pool, so they reach the detection path through host
    memory and PCIe as fetched ARD would.  The runner hands each batch back with
    ``release(batch)`` once its rows are fetched; the pool grows when every buffer is in use.

    mode 'generate': every chip generated on the GPU (DeviceGenerator, one per calling thread; chip
    id = ``chip_of(position)``), its samples written into the pinned batch over PCIe -- exact
    synthetic chips, but the generator's device-to-host traffic shares the link with the uploads
    (the tile-parity run uses it).
    mode 'pool': ``pool_chips`` chips generated once (``prepare``, before a timed run) and every
    position served as a copy of one of them (of the position's own cadence) with its acquisition
    dates moved later by a position-dependent multiple of 16 days (one Landsat repeat cycle, so
    the cadence pattern is kept): every position a distinct (dates, ARD) input whose detection
    genuinely differs (the trend term and the harmonics see other dates), with the statistics of
    a generated chip, produced by host copies at memory speed (``rotate_threads`` per call) and
    without generator traffic on the PCIe link (the bench's tile leg).
    ``generate_seconds`` sums the time spent producing batches."""

    def __init__(self, cfg, device=0, batch_chips=8, n_pix=10000, chip_of=None, pinned=True, mode='generate',
                 pool_chips=64, rotate_threads=8):
        import threading
        self.pinned = pinned
        self.cfg = cfg
        self.device = int(device)
        self.batch_chips = int(batch_chips)
        self.n_pix = int(n_pix)
        self.chip_of = chip_of or (lambda pos: int(pos))
        self.mode = mode
        self.pool_chips = int(pool_chips)
        self.rotate_threads = int(rotate_threads)
        self._local = threading.local()
        self._lock = threading.Lock()
        self._free = []
        self._gens = []
        self._pool = None  # n_obs -> [(chip id, dates, spectra, qa)]
        self.max_obs = max(dates(cfg, c).shape[0] for c in range(64))  # base cadence / sidelap
        self.allocated = 0
        self.generate_seconds = 0.0

    def _gen(self):
        g = getattr(self._local, 'gen', None)
        if g is None:
            g = self._local.gen = DeviceGenerator(self.device)
            with self._lock:
                self._gens.append(g)
        return g

    def prepare(self):
        """'pool' mode: generate the pool chips (ids 0 .. pool_chips-1 of the generator's tile
        range 10^7 + i, by cadence), once."""
        import ccdgpu
        if self.mode != 'pool' or self._pool is not None:
            return
        g = self._gen()
        ids = [10000000 + i for i in range(self.pool_chips)]
        pool = {}
        for i0 in range(0, len(ids), 8):
            b = g.batch(self.cfg, ids[i0:i0 + 8], n_pix=self.n_pix, pinned=False)
            for j, c in enumerate(ids[i0:i0 + 8]):
                d, sp, q = b.chip(j)
                pool.setdefault(int(d.shape[0]), []).append((c, np.array(d), np.array(sp), np.array(q)))
        self._pool = pool

    def _pool_chip(self, pos, chip_id, d):
        """(pool chip, date shift in days) serving position ``pos`` (its chip's dates ``d``)."""
        group = self._pool.get(int(d.shape[0]))
        if not group:
            raise ValueError('no pool chip with %d observations' % d.shape[0])
        h = (int(pos) * 2654435761) & 0xFFFFFFFF
        src = group[h % len(group)]
        if not np.array_equal(src[1], d):
            raise ValueError('pool chip dates differ from the position\'s')
        return src, 16 * (1 + (h >> 8) % 64)

    def __call__(self, positions):
        import time
        import ccdgpu
        t = time.perf_counter()
        g = self._gen() if self.mode == 'generate' else None
        ids = [self.chip_of(p) for p in positions]
        if len(ids) > self.batch_chips:
            raise ValueError('%d chips in one batch, the pool holds %d' % (len(ids), self.batch_chips))
        dts = [g.dates(self.cfg, c) if g is not None else self._dates(c) for c in ids]
        nobs = [d.shape[0] for d in dts]
        if max(nobs) > self.max_obs:
            raise ValueError('chip with %d observations past the pool buffers (%d)' % (max(nobs), self.max_obs))
        with self._lock:
            st = self._free.pop() if self._free else None
            if st is None:
                self.allocated += 1
        if st is None:
            st = ccdgpu.batch_storage(self.batch_chips, self.n_pix, self.max_obs, pinned=self.pinned)
        b = ccdgpu.ChipBatch([self.n_pix] * len(ids), nobs, storage=st)
        if g is not None:
            g.batch(self.cfg, ids, n_pix=self.n_pix, out=b)
        else:
            if self._pool is None:
                raise RuntimeError("TileSource('pool'): call prepare() first")
            for j, (p, c, d) in enumerate(zip(positions, ids, dts)):
                (_, pd, ps, pq), days = self._pool_chip(p, c, d)
                od, os_, oq = b.chip(j)
                od[...] = pd + days
                rotate(ps, pq, 0, os_, oq, self.rotate_threads)  # (shift 0: a parallel copy)
        with self._lock:
            self.generate_seconds += time.perf_counter() - t
        return b

    @property
    def has_views(self):
        return self.mode == 'pool'

    def views(self, positions):
        """'pool' mode without the copy: per position (dates, spectra, qa) where the dates are
        the position's own (moved) acquisition dates and spectra / qa are the pool chip's arrays
        themselves -- for a consumer that makes its own pass over them (ccdc.runner's
        EncodingSource encodes straight from them into pinned memory)."""
        if self.mode != 'pool':
            raise AttributeError('views exist in pool mode only')
        if self._pool is None:
            raise RuntimeError("TileSource('pool'): call prepare() first")
        import time
        t = time.perf_counter()
        out = []
        for p in positions:
            c = self.chip_of(p)
            d = self._dates(c)
            (_, pd, ps, pq), days = self._pool_chip(p, c, d)
            out.append((pd + days, ps, pq))
        with self._lock:
            self.generate_seconds += time.perf_counter() - t
        return out

    def _dates(self, c):
        key = int(c)
        cache = getattr(self, '_date_cache', None)
        if cache is None:
            cache = self._date_cache = {}
        d = cache.get(key)
        if d is None:
            d = cache[key] = dates(self.cfg, key)
        return d

    def release(self, batch):
        if batch.storage is not None:
            with self._lock:
                self._free.append(batch.storage)

    def prefill(self, n):
        """Allocate ``n`` pool buffers ahead (page-locking is slow: keep it out of a timed run)."""
        import ccdgpu
        while self.allocated < n:
            st = ccdgpu.batch_storage(self.batch_chips, self.n_pix, self.max_obs, pinned=self.pinned)
            with self._lock:
                self._free.append(st)
                self.allocated += 1

    def close(self):
        """Close the generators and drop the pool chips and free pinned batches."""
        for g in self._gens:
            g.close()
        self._gens = []
        with self._lock:
            self._free = []
            self._pool = None
