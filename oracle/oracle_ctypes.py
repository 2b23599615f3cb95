"""ctypes loader for oracle/libccdoracle.so (the C restatement).  TEST INFRASTRUCTURE ONLY:
import only from tests/, __graft_entry__.smoke() or bench.py's cpu_baseline leg."""
import ctypes
import os
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(_HERE), 'lcmap-firebird_amd'))
from ccdgpu import abi  # noqa: E402  (struct layouts of include/ccdgpu.h)

_lib = None


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(_HERE, 'libccdoracle.so')
        if not os.path.exists(path):
            raise RuntimeError('oracle not built: make -C oracle')
        L = ctypes.CDLL(path)
        L.ccdoracle_detect_batch.argtypes = [ctypes.POINTER(abi.Params), ctypes.c_int32,
                                             ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.POINTER(abi.Result),
                                             ctypes.c_int32]
        L.ccdoracle_result_free.argtypes = [ctypes.POINTER(abi.Result)]
        L.ccdoracle_chi2_5_ppf.argtypes = [ctypes.c_double]
        L.ccdoracle_chi2_5_ppf.restype = ctypes.c_double
        _lib = L
    return _lib


def detect_batch(dates, spectra, qa, params=None, threads=None):
    """dates [n], spectra [7][n_pix][n] int16, qa [n_pix][n] uint16 -> (rc, abi.Unpacked)."""
    dates = np.ascontiguousarray(dates, dtype=np.int64)
    spectra = np.ascontiguousarray(spectra, dtype=np.int16)
    qa = np.ascontiguousarray(qa, dtype=np.uint16)
    n_pix, n_obs = qa.shape
    assert spectra.shape == (7, n_pix, n_obs) and dates.shape == (n_obs,)
    p = params if isinstance(params, abi.Params) else abi.params_from_dict(params)
    res = abi.Result()
    rc = lib().ccdoracle_detect_batch(ctypes.byref(p), n_pix, n_obs, dates.ctypes.data,
                                      spectra.ctypes.data, qa.ctypes.data, ctypes.byref(res),
                                      int(threads or os.cpu_count() or 1))
    try:
        u = abi.unpack(res)
    finally:
        lib().ccdoracle_result_free(ctypes.byref(res))
    return rc, u
