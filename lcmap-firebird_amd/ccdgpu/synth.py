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
