"""Developer probe (GPU box): round-1's 475ecd7 kernel with EXEC-full checks at every cross-lane
primitive (lib/exp/libr1_475_xl.so, built from `git archive 475ecd7` with the checks added):
prints, per register budget, the first golden case whose run reported a partial-EXEC call site
(CCDGPU_EHIP, 'line 100000 + L')."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'lcmap-firebird_amd'), os.path.join(ROOT, 'tests')]
import numpy as np  # noqa: E402
from ccdgpu import abi  # noqa: E402
import golden_util  # noqa: E402

lib_name, variant = sys.argv[1], sys.argv[2]
os.environ['CCDGPU_KERNEL'] = variant
L = ctypes.CDLL(lib_name)
L.ccdgpu_init.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
L.ccdgpu_detect_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(abi.Params), ctypes.c_int32, ctypes.c_int32,
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(abi.Result)]
L.ccdgpu_result_free.argtypes = [ctypes.POINTER(abi.Result)]
L.ccdgpu_last_error.restype = ctypes.c_char_p
ctx = ctypes.c_void_p()
assert L.ccdgpu_init(0, ctypes.byref(ctx)) == 0
for name in golden_util.names():
    if name == 'dense_daily':
        continue
    (d, s, q), params, ref = golden_util.load(name)
    p = abi.params_from_dict(params)
    d, s, q = (np.ascontiguousarray(x) for x in (d, s, q))
    res = abi.Result()
    rc = L.ccdgpu_detect_batch(ctx, ctypes.byref(p), q.shape[0], q.shape[1], d.ctypes.data, s.ctypes.data,
                               q.ctypes.data, ctypes.byref(res))
    msg = L.ccdgpu_last_error().decode() if rc else ''
    if rc == 0:
        L.ccdgpu_result_free(ctypes.byref(res))
    print(variant, name, rc, msg, flush=True)
