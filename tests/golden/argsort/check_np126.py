"""Pins oracle/ccd_oracle.c's ccdoracle_np_argsort (numpy < 1.17 aquicksort restated) against a
real numpy build's C quicksort: this container's /opt/conda python3.9 carries numpy 1.26.4, whose
baseline (non-SIMD) argsort is the same aquicksort plus the introsort depth limit (not reached by
these inputs); its AVX-512 dispatch (x86-simd-sort, numpy >= 1.25) is switched off with
NPY_DISABLE_CPU_FEATURES, as a pre-2023 numpy would have none.  Run:

  NPY_DISABLE_CPU_FEATURES="AVX512F AVX512CD AVX512_SKX AVX512_CLX AVX512_CNL AVX512_ICL AVX512_SPR" \\
      /opt/conda/bin/python3.9 tests/golden/argsort/check_np126.py

It writes tests/golden/argsort/np126_vectors.npz (inputs and numpy's argsorts) for the CPU suite,
which checks both restatements (C and tests' pure-Python port) against them.
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(HERE)))


def cases(seed=20261018):
    rng = np.random.default_rng(seed)
    out = []
    # closest-DOY keys: |round(d/365.25)*365.25 - d| of real fit-window cadences (multiples of 0.25)
    for n in (17, 24, 25, 40, 64, 100, 257, 700, 1421, 2121):
        for _ in range(6):
            t0 = int(rng.integers(723800, 736000))
            step = rng.choice([1, 7, 8, 16])
            d = np.sort(t0 + np.cumsum(rng.integers(1, 2 * step + 1, n)))
            ref = int(d[int(rng.integers(0, n))]) + int(rng.integers(0, 200))
            drt = (d - ref).astype(np.float64)
            out.append(np.abs(np.round(drt / 365.25) * 365.25 - drt))
    # dates with duplicates, descending as merlin delivers them, and shuffled
    for n in (5, 16, 17, 33, 100, 1000, 2121):
        for _ in range(4):
            d = rng.integers(730000, 730000 + max(2, n // 3), n).astype(np.float64)
            out.append(np.sort(d)[::-1].copy())
            out.append(rng.permutation(d))
    # few distinct values, all equal, sorted runs
    for n in (20, 64, 300):
        out.append(rng.integers(0, 3, n).astype(np.float64))
        out.append(np.zeros(n))
        out.append(np.arange(n, dtype=np.float64))
        out.append(np.arange(n, dtype=np.float64)[::-1].copy())
    return out


def main():
    lib = ctypes.CDLL(os.path.join(ROOT, 'oracle', 'libccdoracle.so'))
    lib.ccdoracle_np_argsort.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                         ctypes.c_void_p]
    from numpy.core._multiarray_umath import __cpu_features__ as f
    simd = [k for k in ('AVX512F', 'AVX512_SKX') if f.get(k)]
    vals, npo, n_mis = [], [], 0
    for v in cases():
        ref = np.argsort(v, kind='quicksort')
        refi = np.argsort(v.astype(np.int64), kind='quicksort') if np.all(v == np.round(v)) else ref
        o = np.arange(v.shape[0], dtype=np.int32)
        lib.ccdoracle_np_argsort(np.ascontiguousarray(v).ctypes.data, o.ctypes.data, v.shape[0], 0, None)
        ok = np.array_equal(o, ref) and np.array_equal(refi, ref)
        n_mis += not ok
        vals.append(v)
        npo.append(ref)
    print('numpy', np.__version__, 'AVX-512 dispatch on:' if simd else 'AVX-512 dispatch off', simd,
          '| cases', len(vals), 'mismatches', n_mis)
    if not simd:
        lens = np.array([v.shape[0] for v in vals])
        np.savez_compressed(os.path.join(HERE, 'np126_vectors.npz'), lens=lens,
                            keys=np.concatenate(vals), argsort=np.concatenate(npo).astype(np.int32),
                            numpy_version=np.array(np.__version__))
    return 1 if (n_mis and not simd) else 0


if __name__ == '__main__':
    sys.exit(main())
