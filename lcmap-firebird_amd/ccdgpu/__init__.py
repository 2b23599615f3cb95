"""ctypes binding of libccdgpu.so (include/ccdgpu.h) -- the MI355X change-detection backend.

This is the only way the Python host side reaches the GPU: plain pointers and sizes through the
C-ABI, no torch types.  The library must be built (``__graft_entry__.build()`` / ``make -C
lcmap-firebird_amd``); if it is missing or no gfx950 device is visible, every call raises
``CcdGpuError`` -- there is no CPU fallback on the product path.
"""
import ctypes
import os
import threading

import numpy as np

from . import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
UPLOAD_SLOTS = 4  # CCDGPU_UPLOAD_SLOTS (include/ccdgpu.h): input slots per context
LIB_PATH = os.environ.get('CCDGPU_LIBRARY') or os.path.join(os.path.dirname(_HERE), 'lib', 'libccdgpu.so')

_lib = None
_lib_lock = threading.Lock()


class CcdGpuError(RuntimeError):
    def __init__(self, code, message):
        super().__init__('ccdgpu error %d: %s' % (code, message))
        self.code = code
        self.message = message


class QAValueError(ValueError):
    """Unsupported bit-packed QA value: the analogue of pyccd qa.qabitval's ValueError."""


def _declare(L):
    c = ctypes
    L.ccdgpu_version.restype = c.c_char_p
    L.ccdgpu_last_error.restype = c.c_char_p
    L.ccdgpu_params_default.argtypes = [c.POINTER(abi.Params)]
    L.ccdgpu_init.argtypes = [c.c_int, c.POINTER(c.c_void_p)]
    if hasattr(L, 'ccdgpu_fetch_batch_rows_into'):
        L.ccdgpu_fetch_batch_rows_into.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p, c.c_int32, c.c_void_p, c.c_int64,
                                                   c.c_void_p, c.c_int64, c.c_void_p, c.c_int64, c.POINTER(c.c_int64)]
        L.ccdgpu_fetch_batch_rows_into.restype = c.c_int
    if hasattr(L, 'ccdgpu_run_slot_begin'):
        L.ccdgpu_run_slot_begin.argtypes = [c.c_void_p, c.c_int32]
        L.ccdgpu_run_slot_begin.restype = c.c_int
        L.ccdgpu_run_query.argtypes = [c.c_void_p]
        L.ccdgpu_run_query.restype = c.c_int
        L.ccdgpu_run_slot_end.argtypes = [c.c_void_p, c.POINTER(c.c_double)]
        L.ccdgpu_run_slot_end.restype = c.c_int
    if hasattr(L, 'ccdgpu_run_slot_begin_rows'):
        L.ccdgpu_run_slot_begin_rows.argtypes = [c.c_void_p, c.c_int32, c.c_void_p, c.c_void_p, c.c_int32, c.c_void_p,
                                                 c.c_int64, c.c_void_p, c.c_int64, c.c_void_p, c.c_int64]
        L.ccdgpu_run_slot_begin_rows.restype = c.c_int
        L.ccdgpu_run_slot_end_rows.argtypes = [c.c_void_p, c.POINTER(c.c_double), c.POINTER(c.c_int64)]
        L.ccdgpu_run_slot_end_rows.restype = c.c_int
    if hasattr(L, 'ccdgpu_init_copy_cus'):
        L.ccdgpu_init_copy_cus.argtypes = [c.c_int, c.c_int, c.POINTER(c.c_void_p)]
        L.ccdgpu_init_copy_cus.restype = c.c_int
    L.ccdgpu_destroy.argtypes = [c.c_void_p]
    L.ccdgpu_device_count.argtypes = [c.POINTER(c.c_int)]
    if hasattr(L, 'ccdgpu_encode_chips'):  # (absent from libraries built before it: A/B runs)
        L.ccdgpu_encoded_bound.argtypes = [c.c_int32, c.c_void_p, c.c_void_p]
        L.ccdgpu_encoded_bound.restype = c.c_int64
        L.ccdgpu_encode_chips.argtypes = [c.c_int32, c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p,
                                          c.c_int64, c.c_int32, c.c_uint16, c.c_uint16]
        L.ccdgpu_encode_chips.restype = c.c_int64
        L.ccdgpu_encode_vector_path.restype = c.c_int32
        L.ccdgpu_stage_slot_encoded.argtypes = [c.c_void_p, c.c_int32, c.c_void_p, c.c_int32, c.c_void_p, c.c_void_p,
                                                c.c_void_p, c.c_void_p, c.c_int64]
        L.ccdgpu_stage_slot_encoded.restype = c.c_int
    if hasattr(L, 'ccdgpu_encoded_check'):
        L.ccdgpu_encoded_check.argtypes = [c.c_int32, c.c_void_p, c.c_void_p, c.c_void_p, c.c_int64]
        L.ccdgpu_encoded_check.restype = c.c_int
    if hasattr(L, 'ccdgpu_device_numa_node'):  # (absent from libraries built before it: A/B runs)
        L.ccdgpu_device_numa_node.argtypes = [c.c_int, c.POINTER(c.c_int)]
        L.ccdgpu_device_numa_node.restype = c.c_int
    L.ccdgpu_synchronize.argtypes = [c.c_void_p]
    L.ccdgpu_detect_batch.argtypes = [c.c_void_p, c.POINTER(abi.Params), c.c_int32, c.c_int32,
                                      c.c_void_p, c.c_void_p, c.c_void_p, c.POINTER(abi.Result)]
    L.ccdgpu_result_free.argtypes = [c.POINTER(abi.Result)]
    L.ccdgpu_stage.argtypes = [c.c_void_p, c.POINTER(abi.Params), c.c_int32, c.c_int32, c.c_int32,
                               c.c_void_p, c.c_void_p, c.c_void_p]
    L.ccdgpu_stage_chips.argtypes = [c.c_void_p, c.POINTER(abi.Params), c.c_int32, c.c_void_p, c.c_void_p,
                                     c.c_void_p, c.c_void_p, c.c_void_p]
    L.ccdgpu_stage_slot_chips.argtypes = [c.c_void_p, c.c_int32, c.POINTER(abi.Params), c.c_int32, c.c_void_p,
                                          c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p]
    L.ccdgpu_fetch_batch_rows.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p, c.c_int32, c.POINTER(abi.Rows)]
    L.ccdgpu_stage_chipmunk.argtypes = [c.c_void_p, c.POINTER(abi.Params), c.c_int32, c.c_int32, c.c_int32,
                                        c.c_void_p, c.c_char_p, c.c_int64, c.c_void_p,
                                        c.POINTER(c.c_double)]
    L.ccdgpu_staged_inputs.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p]
    L.ccdgpu_host_alloc.argtypes = [c.c_size_t, c.POINTER(c.c_void_p)]
    L.ccdgpu_host_free.argtypes = [c.c_void_p]
    L.ccdgpu_stage_slot.argtypes = [c.c_void_p, c.c_int32, c.POINTER(abi.Params), c.c_int32, c.c_int32, c.c_int32,
                                    c.c_void_p, c.c_void_p, c.c_void_p]
    L.ccdgpu_run_slot.argtypes = [c.c_void_p, c.c_int32, c.POINTER(c.c_double)]
    L.ccdgpu_fetch_rows.argtypes = [c.c_void_p, c.c_int32, c.c_int32, c.c_int32, c.c_int32, c.POINTER(abi.Rows)]
    L.ccdgpu_rows_free.argtypes = [c.POINTER(abi.Rows)]
    L.ccdgpu_run_staged.argtypes = [c.c_void_p, c.POINTER(c.c_double)]
    L.ccdgpu_fetch_staged.argtypes = [c.c_void_p, c.c_int32, c.POINTER(abi.Result)]
    L.ccdgpu_last_stats.argtypes = [c.c_void_p, c.POINTER(abi.Stats)]
    L.ccdgpu_diag_counters.argtypes = [c.c_void_p, c.POINTER(c.c_uint64), c.c_int32]
    for name in ('ccdgpu_init', 'ccdgpu_destroy', 'ccdgpu_device_count', 'ccdgpu_synchronize',
                 'ccdgpu_detect_batch', 'ccdgpu_stage', 'ccdgpu_stage_chips', 'ccdgpu_stage_slot_chips',
                 'ccdgpu_fetch_batch_rows', 'ccdgpu_stage_chipmunk', 'ccdgpu_staged_inputs',
                 'ccdgpu_run_staged', 'ccdgpu_fetch_staged', 'ccdgpu_fetch_rows', 'ccdgpu_host_alloc',
                 'ccdgpu_host_free', 'ccdgpu_stage_slot', 'ccdgpu_run_slot', 'ccdgpu_rows_free', 'ccdgpu_fetch_rows',
                 'ccdgpu_last_stats', 'ccdgpu_diag_counters'):
        getattr(L, name).restype = c.c_int
    return L


EXPORTS = ('ccdgpu_version', 'ccdgpu_last_error', 'ccdgpu_params_default', 'ccdgpu_init',
           'ccdgpu_destroy', 'ccdgpu_device_count', 'ccdgpu_synchronize', 'ccdgpu_detect_batch',
           'ccdgpu_result_free', 'ccdgpu_stage', 'ccdgpu_stage_chipmunk', 'ccdgpu_staged_inputs',
           'ccdgpu_run_staged', 'ccdgpu_fetch_staged', 'ccdgpu_fetch_rows', 'ccdgpu_rows_free',
           'ccdgpu_host_alloc', 'ccdgpu_host_free', 'ccdgpu_stage_slot', 'ccdgpu_run_slot',
           'ccdgpu_last_stats', 'ccdgpu_diag_counters', 'ccdgpu_stage_chips', 'ccdgpu_stage_slot_chips',
           'ccdgpu_fetch_batch_rows', 'ccdgpu_device_numa_node', 'ccdgpu_encoded_bound', 'ccdgpu_encode_chips',
           'ccdgpu_encode_vector_path', 'ccdgpu_stage_slot_encoded', 'ccdgpu_init_copy_cus',
           'ccdgpu_run_slot_begin', 'ccdgpu_run_query', 'ccdgpu_run_slot_end', 'ccdgpu_fetch_batch_rows_into',
           'ccdgpu_run_slot_begin_rows', 'ccdgpu_run_slot_end_rows', 'ccdgpu_encoded_check')


def lib():
    """Load libccdgpu.so (raises CcdGpuError if it has not been built)."""
    global _lib
    with _lib_lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise CcdGpuError(abi.E_HIP, 'libccdgpu.so not built at %s (run __graft_entry__.build())' % LIB_PATH)
            _lib = _declare(ctypes.CDLL(LIB_PATH))
    return _lib


def last_error():
    return lib().ccdgpu_last_error().decode()


def _check(rc):
    if rc == abi.E_QA:
        raise QAValueError(last_error())
    if rc != 0:
        raise CcdGpuError(rc, last_error())


def version():
    return lib().ccdgpu_version().decode()


def device_count():
    n = ctypes.c_int(0)
    rc = lib().ccdgpu_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0


def device_numa_node(device=0):
    """NUMA node the GPU ``device`` is attached to (-1: not exposed by the platform)."""
    n = ctypes.c_int(-1)
    _check(lib().ccdgpu_device_numa_node(int(device), ctypes.byref(n)))
    return n.value


def default_params():
    p = abi.Params()
    lib().ccdgpu_params_default(ctypes.byref(p))
    return p


class ChipBatch(object):
    """Host buffers of one staged batch in the ccdgpu_stage_chips layout (include/ccdgpu.h):
    chips of their own pixel / observation counts packed back to back.  ``pinned=True``
    allocates them in page-locked memory (ccdgpu_host_alloc) so uploads overlap detection.

        b = ChipBatch([10000, 10000], [1421, 2121], pinned=True)
        d, s, q = b.chip(1)      # views: dates [n], spectra [7][n_pix][n], qa [n_pix][n]
    """

    def __init__(self, n_pix, n_obs, pinned=False, storage=None):
        """``storage``: (dates int64, spectra int16, qa uint16) 1-D arrays of at least the batch's
        sizes (e.g. ``batch_storage``, reused across batches): the batch's arrays are their
        prefixes instead of new allocations."""
        self.n_pix = np.ascontiguousarray(n_pix, dtype=np.int32).reshape(-1)
        self.n_obs = np.ascontiguousarray(n_obs, dtype=np.int32).reshape(-1)
        if self.n_pix.shape != self.n_obs.shape or self.n_pix.size == 0:
            raise ValueError('n_pix and n_obs must be equal-length, non-empty')
        self.obs_off = np.concatenate([[0], np.cumsum(self.n_obs, dtype=np.int64)])
        self.pix_off = np.concatenate([[0], np.cumsum(self.n_pix, dtype=np.int64)])
        self.data_off = np.concatenate([[0], np.cumsum(self.n_pix.astype(np.int64) * self.n_obs)])
        nd, ns = int(self.obs_off[-1]), int(self.data_off[-1])
        self.storage = storage
        if storage is not None:
            sd, ss, sq = storage
            if sd.dtype != np.int64 or ss.dtype != np.int16 or sq.dtype != np.uint16 or \
                    sd.size < nd or ss.size < 7 * ns or sq.size < ns:
                raise ValueError('storage too small or of the wrong types for this batch')
            self.dates, self.spectra, self.qa = sd[:nd], ss[:7 * ns], sq[:ns]
            return
        alloc = pinned_empty if pinned else np.empty
        self.dates = alloc((nd,), np.int64)
        self.spectra = alloc((7 * ns,), np.int16)
        self.qa = alloc((ns,), np.uint16)

    @property
    def n_chips(self):
        return int(self.n_pix.size)

    @property
    def total_pixels(self):
        return int(self.pix_off[-1])

    @property
    def nbytes(self):
        return self.dates.nbytes + self.spectra.nbytes + self.qa.nbytes

    def chip(self, c):
        """Views of chip c: (dates [n], spectra [7][n_pix][n], qa [n_pix][n])."""
        npx, n = int(self.n_pix[c]), int(self.n_obs[c])
        o, d = int(self.obs_off[c]), int(self.data_off[c])
        return (self.dates[o:o + n], self.spectra[7 * d:7 * (d + npx * n)].reshape(7, npx, n),
                self.qa[d:d + npx * n].reshape(npx, n))

    def set_chip(self, c, dates, spectra, qa):
        d, s, q = self.chip(c)
        d[...], s[...], q[...] = dates, spectra, qa

    @classmethod
    def from_chips(cls, chips, pinned=False):
        """[(dates [n], spectra [7][n_pix][n], qa [n_pix][n]), ...] -> ChipBatch."""
        chips = list(chips)
        b = cls([c[2].shape[0] for c in chips], [c[0].shape[0] for c in chips], pinned=pinned)
        for i, (d, s, q) in enumerate(chips):
            b.set_chip(i, d, s, q)
        return b

    def mask_of(self, bits, c):
        """Chip c's int8 [n_pix][n_obs] processing mask from a batch row fetch's bit words."""
        p0, p1 = int(self.pix_off[c]), int(self.pix_off[c + 1])
        return abi.unpack_mask_bits(bits[p0:p1], int(self.n_obs[c]))

    def mask_bits_of(self, bits, c):
        """Chip c's bit words of a batch row fetch, [n_pix][ceil(n_obs / 32)] (no unpacking;
        the batch's own word count, set by its largest chip, is trimmed to the chip's)."""
        return bits[int(self.pix_off[c]):int(self.pix_off[c + 1]), :(int(self.n_obs[c]) + 31) // 32]


class EncodedBatch(ChipBatch):
    """A batch in the transport encoding of ccdgpu_encode_chips (include/ccdgpu.h): the chips'
    dates plus one byte buffer, uploaded with Context.stage_slot_encoded and decoded on the device
    into the ChipBatch layout.  Shape, dates and mask helpers as ChipBatch; chip(c) gives
    (dates, None, None) -- the pixel data exist only in encoded form.

        e = EncodedBatch.encode([(d0, s0, q0), (d1, s1, q1)], storage=encode_storage(...))
    """

    def __init__(self, n_pix, n_obs, storage=None, pinned=True):
        self.n_pix = np.ascontiguousarray(n_pix, dtype=np.int32).reshape(-1)
        self.n_obs = np.ascontiguousarray(n_obs, dtype=np.int32).reshape(-1)
        if self.n_pix.shape != self.n_obs.shape or self.n_pix.size == 0:
            raise ValueError('n_pix and n_obs must be equal-length, non-empty')
        self.obs_off = np.concatenate([[0], np.cumsum(self.n_obs, dtype=np.int64)])
        self.pix_off = np.concatenate([[0], np.cumsum(self.n_pix, dtype=np.int64)])
        self.data_off = np.concatenate([[0], np.cumsum(self.n_pix.astype(np.int64) * self.n_obs)])
        bound = int(lib().ccdgpu_encoded_bound(self.n_chips, self.n_pix.ctypes.data, self.n_obs.ctypes.data))
        nd = int(self.obs_off[-1])
        self.storage = storage
        if storage is not None:
            sd, sb = storage
            if sd.dtype != np.int64 or sb.dtype != np.uint8 or sd.size < nd or sb.size < bound:
                raise ValueError('storage too small or of the wrong types for this batch')
            self.dates, self.buf = sd[:nd], sb
        else:
            alloc = pinned_empty if pinned else np.empty
            self.dates, self.buf = alloc((nd,), np.int64), alloc((bound,), np.uint8)
        self.spectra = self.qa = None
        self.bound = bound
        self.nbytes_encoded = 0

    @property
    def nbytes(self):
        return self.dates.nbytes + self.nbytes_encoded

    def chip(self, c):
        n, o = int(self.n_obs[c]), int(self.obs_off[c])
        return self.dates[o:o + n], None, None

    def set_chip(self, c, dates, spectra, qa):
        raise TypeError('EncodedBatch holds encoded chips: build it with EncodedBatch.encode')

    def fill(self, chips, threads=4, drop_bits=1, strict_bits=1):
        """Encode chips [(dates [n], spectra [7][n_pix][n] int16, qa [n_pix][n] uint16), ...]
        (any C-contiguous arrays: pinned batch views, or a source's own arrays -- nothing else is
        copied) into this batch; returns the encoded bytes.  ``drop_bits`` / ``strict_bits``:
        QA bits whose observations send no band values / must hold -9999 (include/ccdgpu.h; the
        default, the fill bit for both, is lossless; ``unread_drop_bits(params)`` gives the bits of
        observations the detection never reads)."""
        chips = list(chips)
        if len(chips) != self.n_chips:
            raise ValueError('%d chips for a batch of %d' % (len(chips), self.n_chips))
        sp = (ctypes.c_void_p * len(chips))()
        qp = (ctypes.c_void_p * len(chips))()
        keep = []
        for i, (d, s, q) in enumerate(chips):
            d = np.asarray(d)
            s = np.ascontiguousarray(s, dtype=np.int16)
            q = np.ascontiguousarray(q, dtype=np.uint16)
            if d.shape != (int(self.n_obs[i]),) or s.shape != (7, int(self.n_pix[i]), int(self.n_obs[i])) or \
                    q.shape != (int(self.n_pix[i]), int(self.n_obs[i])):
                raise ValueError('chip %d does not have this batch\'s shape' % i)
            o = int(self.obs_off[i])
            self.dates[o:o + d.shape[0]] = d
            sp[i], qp[i] = s.ctypes.data, q.ctypes.data
            keep.append((s, q))
        n = int(lib().ccdgpu_encode_chips(self.n_chips, self.n_pix.ctypes.data, self.n_obs.ctypes.data,
                                          ctypes.cast(sp, ctypes.c_void_p), ctypes.cast(qp, ctypes.c_void_p),
                                          self.buf.ctypes.data, self.buf.size, int(threads), int(drop_bits),
                                          int(strict_bits)))
        if n < 0:
            raise ValueError('ccdgpu_encode_chips failed (%d)' % n)
        self.nbytes_encoded = n
        return n

    @classmethod
    def encode(cls, chips, threads=4, storage=None, pinned=True, drop_bits=1, strict_bits=1):
        chips = list(chips)
        b = cls([c[2].shape[0] for c in chips], [c[0].shape[0] for c in chips], storage=storage, pinned=pinned)
        b.fill(chips, threads, drop_bits, strict_bits)
        return b

    def check(self):
        """The header / layout checks of the upload (ccdgpu_encoded_check; no device needed):
        raises CcdGpuError naming the first problem."""
        _check(lib().ccdgpu_encoded_check(self.n_chips, self.n_pix.ctypes.data, self.n_obs.ctypes.data,
                                          self.buf.ctypes.data, int(self.nbytes_encoded)))

    def chip_modes(self):
        """Per chip: 1 if encoded, 0 if sent raw (from the section headers)."""
        off = self.buf[8:8 * (self.n_chips + 2)].view(np.int64)
        return [int(self.buf[int(o):int(o) + 4].view(np.int32)[0]) for o in off[:self.n_chips]]


def encode_storage(max_chips, max_pix, max_obs, pinned=True):
    """Reusable buffers for EncodedBatch(..., storage=...): room for ``max_chips`` chips of up to
    ``max_pix`` pixels x ``max_obs`` observations."""
    n = int(max_chips)
    np_ = np.full(n, int(max_pix), dtype=np.int32)
    no = np.full(n, int(max_obs), dtype=np.int32)
    bound = int(lib().ccdgpu_encoded_bound(n, np_.ctypes.data, no.ctypes.data))
    alloc = pinned_empty if pinned else np.empty
    return alloc((n * int(max_obs),), np.int64), alloc((bound,), np.uint8)


def unread_drop_bits(params=None):
    """(drop_bits, strict_bits) for the transport encoding that drops every band value the
    detection never reads: observations whose QA word has the fill, cloud or shadow bit (qabitval
    classes them as fill / cloud / shadow whatever else is set, and no procedure keeps those
    classes); fill observations stay strict (their bands must be -9999).  For non-bit-packed QA
    (class values, not bits) only the lossless (fill bit 0) setting applies."""
    p = params if isinstance(params, abi.Params) else abi.params_from_dict(params)
    if not p.qa_bitpacked:
        return 0, 0
    bits = [int(p.qa_fill), int(p.qa_cloud), int(p.qa_shadow)]
    if any(b < 0 or b > 15 for b in bits):
        return 0, 0  # (bits outside a 16-bit word: nothing dropped)
    drop = 0
    for b in bits:
        drop |= 1 << b
    return drop, 1 << int(p.qa_fill)


def encode_vector_path():
    """True if the encoder uses AVX-512 VBMI2 compress-stores on this CPU."""
    return bool(lib().ccdgpu_encode_vector_path())


def _as_inputs(dates, spectra, qa):
    dates = np.ascontiguousarray(dates, dtype=np.int64)
    spectra = np.ascontiguousarray(spectra, dtype=np.int16)
    qa = np.ascontiguousarray(qa, dtype=np.uint16)
    return dates, spectra, qa


class Context(object):
    """One HIP device + stream (ccdgpu_ctx).  Not shared across threads."""

    def __init__(self, device=0, copy_cus=0):
        """copy_cus > 0 reserves that many CUs for the context's copy stream (upload decode,
        blits), the rest for detection (ccdgpu_init_copy_cus, include/ccdgpu.h)."""
        self.qa_error = False
        self._ctx = ctypes.c_void_p()
        L = lib()
        if copy_cus and hasattr(L, 'ccdgpu_init_copy_cus'):
            _check(L.ccdgpu_init_copy_cus(int(device), int(copy_cus), ctypes.byref(self._ctx)))
        else:
            _check(L.ccdgpu_init(int(device), ctypes.byref(self._ctx)))
        self.device = device

    def close(self):
        if self._ctx:
            lib().ccdgpu_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def synchronize(self):
        _check(lib().ccdgpu_synchronize(self._ctx))

    def detect_batch(self, dates, spectra, qa, params=None):
        """Pixels sharing one date vector: dates [n], spectra [7][n_pix][n], qa [n_pix][n].
        Returns abi.Unpacked.  Raises QAValueError on unsupported QA values."""
        dates, spectra, qa = _as_inputs(dates, spectra, qa)
        n_pix, n_obs = qa.shape
        if spectra.shape != (7, n_pix, n_obs) or dates.shape != (n_obs,):
            raise ValueError('shape mismatch: dates %s spectra %s qa %s' % (dates.shape, spectra.shape, qa.shape))
        p = params if isinstance(params, abi.Params) else abi.params_from_dict(params)
        res = abi.Result()
        rc = lib().ccdgpu_detect_batch(self._ctx, ctypes.byref(p), n_pix, n_obs, dates.ctypes.data,
                                       spectra.ctypes.data, qa.ctypes.data, ctypes.byref(res))
        try:
            if rc not in (0, abi.E_QA):
                _check(rc)
            u = abi.unpack(res)
        finally:
            lib().ccdgpu_result_free(ctypes.byref(res))
        if rc == abi.E_QA:
            err = QAValueError(last_error())
            err.result = u
            raise err
        return u

    # device-resident path ------------------------------------------------------------------
    def stage(self, dates, spectra, qa, params=None):
        """dates [C][n], spectra [C][7][n_pix][n], qa [C][n_pix][n] -> staged on the device."""
        dates, spectra, qa = _as_inputs(dates, spectra, qa)
        n_chips, n_pix, n_obs = qa.shape
        p = params if isinstance(params, abi.Params) else abi.params_from_dict(params)
        _check(lib().ccdgpu_stage(self._ctx, ctypes.byref(p), n_chips, n_pix, n_obs,
                                  dates.ctypes.data, spectra.ctypes.data, qa.ctypes.data))
        self._keep = (dates, spectra, qa)
        self._n_pix = n_pix

    def stage_chips(self, batch, params=None):
        """Stage a ChipBatch (or a list of (dates, spectra, qa) chips of any sizes) in one
        batch: ccdgpu_stage_chips."""
        if not isinstance(batch, ChipBatch):
            batch = ChipBatch.from_chips(batch)
        p = params if isinstance(params, abi.Params) else abi.params_from_dict(params)
        _check(lib().ccdgpu_stage_chips(self._ctx, ctypes.byref(p), batch.n_chips, batch.n_pix.ctypes.data,
                                        batch.n_obs.ctypes.data, batch.dates.ctypes.data,
                                        batch.spectra.ctypes.data, batch.qa.ctypes.data))
        self._keep = batch
        self._n_pix = None
        return batch

    def stage_slot_chips(self, slot, batch, params=None):
        """Upload a ChipBatch into input slot 0 .. UPLOAD_SLOTS-1 on the copy stream and return at once (the
        batch must stay alive and unchanged until run_slot(slot) returns; pinned=True batches
        upload asynchronously).  An EncodedBatch goes through stage_slot_encoded."""
        if isinstance(batch, EncodedBatch):
            return self.stage_slot_encoded(slot, batch, params)
        p = params if isinstance(params, abi.Params) else abi.params_from_dict(params)
        _check(lib().ccdgpu_stage_slot_chips(self._ctx, int(slot), ctypes.byref(p), batch.n_chips,
                                             batch.n_pix.ctypes.data, batch.n_obs.ctypes.data,
                                             batch.dates.ctypes.data, batch.spectra.ctypes.data,
                                             batch.qa.ctypes.data))
        if not hasattr(self, '_slot_keep'):
            self._slot_keep = {}
        self._slot_keep[int(slot)] = batch

    def stage_slot_encoded(self, slot, batch, params=None):
        """Upload an EncodedBatch into input slot ``slot`` and decode it there on the device (copy
        stream; same life-time rules as stage_slot_chips)."""
        p = params if isinstance(params, abi.Params) else abi.params_from_dict(params)
        _check(lib().ccdgpu_stage_slot_encoded(self._ctx, int(slot), ctypes.byref(p), batch.n_chips,
                                               batch.n_pix.ctypes.data, batch.n_obs.ctypes.data,
                                               batch.dates.ctypes.data, batch.buf.ctypes.data,
                                               int(batch.nbytes_encoded)))
        if not hasattr(self, '_slot_keep'):
            self._slot_keep = {}
        self._slot_keep[int(slot)] = batch

    def fetch_batch_rows(self, cx, cy, width=100):
        """Rows of every chip of the last run in one device pass and one copy: (row_offsets
        [total_pixels+1], rows abi.ROW_DTYPE, mask bit words uint32 [total_pixels][words] --
        ChipBatch.mask_of(bits, c) is chip c's int8 [n_pix][n_obs] mask)."""
        batch = self._keep
        if not isinstance(batch, ChipBatch):
            raise ValueError('fetch_batch_rows needs a stage_chips / stage_slot_chips batch')
        cx = np.ascontiguousarray(cx, dtype=np.int32)
        cy = np.ascontiguousarray(cy, dtype=np.int32)
        if cx.shape != (batch.n_chips,) or cy.shape != (batch.n_chips,):
            raise ValueError('cx / cy need one entry per chip (%d)' % batch.n_chips)
        r = abi.Rows()
        rc = lib().ccdgpu_fetch_batch_rows(self._ctx, cx.ctypes.data, cy.ctypes.data, int(width), ctypes.byref(r))
        try:
            _check(rc)
            return abi.unpack_rows(r)
        finally:
            lib().ccdgpu_rows_free(ctypes.byref(r))

    def fetch_batch_rows_into(self, cx, cy, bufs, width=100):
        """fetch_batch_rows into ``bufs`` (a RowsBuffers, reused across batches: pinned, so the
        rows and mask words arrive by DMA with no host copy; ccdgpu_fetch_batch_rows_into).
        Returns views of its arrays, valid until its next use."""
        batch = self._keep
        if not isinstance(batch, ChipBatch):
            raise ValueError('fetch_batch_rows needs a stage_chips / stage_slot_chips batch')
        cx = np.ascontiguousarray(cx, dtype=np.int32)
        cy = np.ascontiguousarray(cy, dtype=np.int32)
        if cx.shape != (batch.n_chips,) or cy.shape != (batch.n_chips,):
            raise ValueError('cx / cy need one entry per chip (%d)' % batch.n_chips)
        L = lib()
        if not hasattr(L, 'ccdgpu_fetch_batch_rows_into'):  # (libraries built before it: A/B runs)
            return self.fetch_batch_rows(cx, cy, width)
        n_pix = int(batch.pix_off[-1])
        words = (int(batch.n_obs.max()) + 31) // 32
        bufs.ensure(n_pix + 1, n_pix * 2, n_pix * words)
        nr = ctypes.c_int64(0)
        for _ in range(2):
            rc = L.ccdgpu_fetch_batch_rows_into(self._ctx, cx.ctypes.data, cy.ctypes.data, int(width),
                                                bufs.offsets.ctypes.data, bufs.offsets.size, bufs.rows.ctypes.data,
                                                bufs.rows.size, bufs.mask.ctypes.data, bufs.mask.size, ctypes.byref(nr))
            if rc == 0:
                break
            if rc != abi.E_INVAL or nr.value <= bufs.rows.size:
                _check(rc)
            bufs.ensure(n_pix + 1, nr.value, n_pix * words)  # more rows than the first guess
        else:
            _check(rc)
        return bufs.offsets[:n_pix + 1], bufs.rows[:nr.value], bufs.mask[:n_pix * words].reshape(n_pix, words)

    def stage_slot(self, slot, dates, spectra, qa, params=None):
        """Upload a batch into input slot 0 .. UPLOAD_SLOTS-1 on the copy stream and return at once (the arrays
        must stay alive and unchanged until run_slot(slot) returns; pinned arrays from
        ``pinned_empty`` make the upload overlap a running detection)."""
        dates, spectra, qa = _as_inputs(dates, spectra, qa)
        n_chips, n_pix, n_obs = qa.shape
        p = params if isinstance(params, abi.Params) else abi.params_from_dict(params)
        _check(lib().ccdgpu_stage_slot(self._ctx, int(slot), ctypes.byref(p), n_chips, n_pix, n_obs,
                                       dates.ctypes.data, spectra.ctypes.data, qa.ctypes.data))
        if not hasattr(self, '_slot_keep'):
            self._slot_keep = {}
        self._slot_keep[int(slot)] = (dates, spectra, qa)

    def run_slot(self, slot):
        """Detect the batch of input slot ``slot`` (waits for its upload); fetch / fetch_rows as
        after run().  Returns the kernel seconds."""
        secs = ctypes.c_double(0.0)
        rc = lib().ccdgpu_run_slot(self._ctx, int(slot), ctypes.byref(secs))
        if rc not in (0, abi.E_QA):
            _check(rc)
        self.qa_error = rc == abi.E_QA  # results exist; the pixel's procedure is -1 (fetch)
        self._keep = self._slot_keep.get(int(slot))
        self._n_pix = None if isinstance(self._keep, ChipBatch) else self._keep[2].shape[1]
        return secs.value

    def run_slot_begin(self, slot):
        """run_slot in halves (ccdgpu_run_slot_begin / _query / _end): launch the detection of
        slot ``slot`` and return at once; run_done() says whether it has completed, and
        run_slot_end() waits for it and finishes as run_slot does.  In between, only stage_slot*
        of other slots may be called."""
        _check(lib().ccdgpu_run_slot_begin(self._ctx, int(slot)))
        self._pending_slot = int(slot)

    def run_done(self):
        rc = lib().ccdgpu_run_query(self._ctx)
        if rc < 0:
            _check(rc)
        return rc == 1

    def run_slot_begin_rows(self, slot, cx, cy, bufs, width=100):
        """run_slot_begin with the batch's rows in the same device chain
        (ccdgpu_run_slot_begin_rows): chip c's rows at (cx[c], cy[c]) land in ``bufs`` (a
        RowsBuffers, grown here to the slot's pixels: offsets, mask words, and rows for
        ``rows_per_pixel`` per pixel); run_slot_end_rows() waits once and returns them."""
        batch = self._slot_keep.get(int(slot)) if hasattr(self, '_slot_keep') else None
        if not isinstance(batch, ChipBatch):
            raise ValueError('run_slot_begin_rows needs a stage_slot_chips / stage_slot_encoded batch')
        cx = np.ascontiguousarray(cx, dtype=np.int32)
        cy = np.ascontiguousarray(cy, dtype=np.int32)
        if cx.shape != (batch.n_chips,) or cy.shape != (batch.n_chips,):
            raise ValueError('cx / cy need one entry per chip (%d)' % batch.n_chips)
        n_pix = int(batch.pix_off[-1])
        words = (int(batch.n_obs.max()) + 31) // 32
        bufs.ensure(n_pix + 1, int(bufs.rows_per_pixel * n_pix) + 64, n_pix * words)
        rate = bufs.copy_per_pixel if bufs.copy_per_pixel is not None else bufs.rows_per_pixel
        cap = min(bufs.rows.size, int(rate * n_pix) + 64)
        _check(lib().ccdgpu_run_slot_begin_rows(self._ctx, int(slot), cx.ctypes.data, cy.ctypes.data, int(width),
                                                bufs.offsets.ctypes.data, bufs.offsets.size, bufs.rows.ctypes.data,
                                                cap, bufs.mask.ctypes.data, bufs.mask.size))
        self._pending_slot = int(slot)
        self._rows_req = (cx, cy, bufs, int(width), n_pix, words, cap)

    def run_slot_end_rows(self):
        """(row_offsets [n_pix+1], rows, mask words [n_pix][words]) of the batch begun with
        run_slot_begin_rows -- views of its RowsBuffers, valid until their next use.  More rows
        than the buffer held: the buffer grows (and learns the rate) and the rows are fetched."""
        secs = ctypes.c_double(0.0)
        nr = ctypes.c_int64(0)
        rc = lib().ccdgpu_run_slot_end_rows(self._ctx, ctypes.byref(secs), ctypes.byref(nr))
        cx, cy, bufs, width, n_pix, words, cap = self._rows_req
        self._rows_req = None
        self._keep = self._slot_keep.get(self._pending_slot)
        self._n_pix = None
        if nr.value > 0:
            bufs.max_rate = max(bufs.max_rate, nr.value / max(1, n_pix))
            bufs.copy_per_pixel = min(bufs.rows_per_pixel, 1.25 * bufs.max_rate)
        short = (rc == abi.E_OVERFLOW and 'rows' in last_error()) or rc == abi.E_QA
        if short and nr.value > cap and self._keep is not None:
            # the run is complete but its rows did not fit: grow, learn the rate, fetch them (an
            # unsupported QA value comes back as E_QA with the count set, and still raises)
            bufs.rows_per_pixel = max(bufs.rows_per_pixel, 1.25 * nr.value / max(1, n_pix))
            bufs.copy_per_pixel = min(bufs.rows_per_pixel, 1.25 * bufs.max_rate)
            self.qa_error = rc == abi.E_QA
            return self.fetch_batch_rows_into(cx, cy, bufs, width)
        if rc not in (0, abi.E_QA):
            _check(rc)
        self.qa_error = rc == abi.E_QA
        n = nr.value
        return bufs.offsets[:n_pix + 1], bufs.rows[:n], bufs.mask[:n_pix * words].reshape(n_pix, words)

    def run_slot_end(self):
        secs = ctypes.c_double(0.0)
        rc = lib().ccdgpu_run_slot_end(self._ctx, ctypes.byref(secs))
        if rc not in (0, abi.E_QA):
            _check(rc)
        self.qa_error = rc == abi.E_QA
        slot = self._pending_slot
        self._keep = self._slot_keep.get(slot)
        self._n_pix = None if isinstance(self._keep, ChipBatch) else self._keep[2].shape[1]
        return secs.value

    def stage_chipmunk(self, dates, text, offsets, n_pix, params=None):
        """Stage chips from the chipmunk wire format (see ccdc.chipmunk.pack_text):
        dates [C][n] int64, text bytes (concatenated base64 payloads), offsets [C][n][8] int64
        byte offsets of each layer's payload (-1 = missing layer).  Decoding and the pivot to
        the detection layout run on the device; returns the unpack kernel time in seconds."""
        dates = np.ascontiguousarray(dates, dtype=np.int64)
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        if dates.ndim == 1:
            dates = dates[None]
        if offsets.ndim == 2:
            offsets = offsets[None]
        n_chips, n_obs = dates.shape
        if offsets.shape != (n_chips, n_obs, 8):
            raise ValueError('offsets must be [n_chips][n_obs][8], got %r' % (offsets.shape,))
        text = bytes(text)
        p = params if isinstance(params, abi.Params) else abi.params_from_dict(params)
        secs = ctypes.c_double(0.0)
        _check(lib().ccdgpu_stage_chipmunk(self._ctx, ctypes.byref(p), n_chips, int(n_pix), n_obs,
                                           dates.ctypes.data, text, len(text), offsets.ctypes.data,
                                           ctypes.byref(secs)))
        self._keep = (dates, text, offsets)
        self._n_pix = int(n_pix)
        return secs.value

    def staged_inputs(self):
        """The staged pixel inputs copied back: (spectra [C][7][n_pix][n], qa [C][n_pix][n]) for
        a uniform batch, flat (spectra, qa) in the ChipBatch layout for a stage_chips batch."""
        if isinstance(self._keep, ChipBatch):  # (an EncodedBatch too: decoded on the device)
            b = self._keep
            nd = int(b.data_off[-1])
            spectra, qa = np.empty(7 * nd, dtype=np.int16), np.empty(nd, dtype=np.uint16)
            _check(lib().ccdgpu_staged_inputs(self._ctx, spectra.ctypes.data, qa.ctypes.data))
            return spectra, qa
        d = self._keep[0]
        n_chips, n_obs = d.shape if d.ndim == 2 else (1, d.shape[0])
        n_pix = self._n_pix
        spectra = np.empty((n_chips, 7, n_pix, n_obs), dtype=np.int16)
        qa = np.empty((n_chips, n_pix, n_obs), dtype=np.uint16)
        _check(lib().ccdgpu_staged_inputs(self._ctx, spectra.ctypes.data, qa.ctypes.data))
        return spectra, qa

    def run(self):
        secs = ctypes.c_double(0.0)
        rc = lib().ccdgpu_run_staged(self._ctx, ctypes.byref(secs))
        if rc not in (0, abi.E_QA):
            _check(rc)
        self.qa_error = rc == abi.E_QA  # results exist; the pixel's procedure is -1 (fetch)
        return secs.value

    def fetch(self, chip):
        res = abi.Result()
        rc = lib().ccdgpu_fetch_staged(self._ctx, int(chip), ctypes.byref(res))
        try:
            _check(rc)
            return abi.unpack(res)
        finally:
            lib().ccdgpu_result_free(ctypes.byref(res))

    def fetch_rows(self, chip, cx, cy, width=100):
        """Segment / pixel table rows of staged chip ``chip`` (output writer, packed on the
        device): (row_offsets [n_pix+1], rows abi.ROW_DTYPE [n_rows], mask int8 [n_pix][n_obs])."""
        r = abi.Rows()
        rc = lib().ccdgpu_fetch_rows(self._ctx, int(chip), int(cx), int(cy), int(width), ctypes.byref(r))
        try:
            _check(rc)
            return abi.unpack_rows(r)
        finally:
            lib().ccdgpu_rows_free(ctypes.byref(r))

    def diag_counters(self):
        buf = (ctypes.c_uint64 * 48)()
        _check(lib().ccdgpu_diag_counters(self._ctx, buf, 48))
        return list(buf)

    def stats(self):
        s = abi.Stats()
        _check(lib().ccdgpu_last_stats(self._ctx, ctypes.byref(s)))
        return {k: getattr(s, k) for k, _ in abi.Stats._fields_}


class _Pinned(object):
    """Owner of one ccdgpu_host_alloc block (freed when the last array view goes away)."""
    def __init__(self, nbytes):
        self.ptr = ctypes.c_void_p()
        _check(lib().ccdgpu_host_alloc(int(nbytes), ctypes.byref(self.ptr)))
        self.nbytes = int(nbytes)

    def __del__(self):
        try:
            if self.ptr:
                lib().ccdgpu_host_free(self.ptr)
        except Exception:
            pass


def batch_storage(max_chips, max_pix, max_obs, pinned=True):
    """Reusable buffers for ChipBatch(..., storage=...): room for ``max_chips`` chips of up to
    ``max_pix`` pixels x ``max_obs`` observations."""
    alloc = pinned_empty if pinned else np.empty
    n = int(max_chips) * int(max_pix) * int(max_obs)
    return (alloc((int(max_chips) * int(max_obs),), np.int64), alloc((7 * n,), np.int16), alloc((n,), np.uint16))


class RowsBuffers(object):
    """Reusable (pinned) landing buffers of Context.fetch_batch_rows_into: row offsets, rows
    (abi.ROW_DTYPE) and mask words; grown on demand, 25 % headroom."""

    def __init__(self, pinned=True, rows_per_pixel=2.0):
        self.pinned = pinned
        self.rows_per_pixel = float(rows_per_pixel)  # rows room of a batch chain (run_slot_begin_rows)
        # rows a batch chain copies back per pixel: learned from the batches seen (1.25 x the
        # highest rate, at most rows_per_pixel), so the copy is not the whole room -- a tile of
        # ~1 row per pixel copies ~1.25 instead of 2 rows' bytes per pixel; a batch with more
        # rows than that takes the rows-overflow path once and raises the rate
        self.copy_per_pixel = None
        self.max_rate = 0.0
        self.offsets = np.zeros(0, np.int64)
        self.rows = np.zeros(0, abi.ROW_DTYPE)
        self.mask = np.zeros(0, np.uint32)

    def _grow(self, arr, n, dtype):
        if arr.size >= n:
            return arr
        n = int(n * 1.25) + 64
        return pinned_empty((n,), dtype) if self.pinned else np.empty(n, dtype)

    def ensure(self, n_offsets, n_rows, n_words):
        self.offsets = self._grow(self.offsets, n_offsets, np.int64)
        self.rows = self._grow(self.rows, n_rows, abi.ROW_DTYPE)
        self.mask = self._grow(self.mask, n_words, np.uint32)


def pinned_empty(shape, dtype):
    """numpy array in pinned (page-locked) host memory: uploads from it are asynchronous."""
    dtype = np.dtype(dtype)
    n = int(np.prod(shape)) * dtype.itemsize
    owner = _Pinned(n)
    buf = (ctypes.c_char * max(n, 1)).from_address(owner.ptr.value)
    arr = np.frombuffer(buf, dtype=dtype, count=int(np.prod(shape))).reshape(shape)
    return _PinnedArray(arr, owner)


class _PinnedArray(np.ndarray):
    """ndarray view whose base keeps the pinned allocation alive."""
    def __new__(cls, arr, owner):
        obj = np.asarray(arr).view(cls)
        obj._pinned_owner = owner
        return obj

    def __array_finalize__(self, obj):
        if obj is not None:
            self._pinned_owner = getattr(obj, '_pinned_owner', None)


_default_ctx = {}


def default_context(device=None):
    """Per-thread default context on ``device`` (HIP_VISIBLE_DEVICES-relative, default 0)."""
    if device is None:
        device = int(os.environ.get('CCDGPU_DEVICE', '0'))
    key = (threading.get_ident(), device)
    ctx = _default_ctx.get(key)
    if ctx is None:
        ctx = Context(device)
        _default_ctx[key] = ctx
    return ctx
