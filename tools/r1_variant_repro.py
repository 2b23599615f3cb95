"""Developer probe (GPU box): the round-1 kernel at commit 475ecd7 -- where the 4-waves/SIMD (w4)
build was recorded as breaking golden parity -- rebuilt with a w4 variant twice, with HIP's
default fp contraction and with -ffp-contract=on (lib/libr1_475_fast.so / _on.so, built from
`git archive 475ecd7`).  For each library and register budget: golden problems, and whether the
results are byte-identical to that library's w3.  Round-1 C-ABI through raw ctypes."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'lcmap-firebird_amd'), os.path.join(ROOT, 'tests')]
from ccdgpu import abi  # noqa: E402
import golden_util, parity_util  # noqa: E402


def run(lib_name, variant):
    os.environ['CCDGPU_KERNEL'] = variant
    L = ctypes.CDLL(lib_name if os.path.isabs(lib_name) else os.path.join(ROOT, 'lcmap-firebird_amd', 'lib', lib_name))
    L.ccdgpu_init.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    L.ccdgpu_detect_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(abi.Params), ctypes.c_int32, ctypes.c_int32,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(abi.Result)]
    L.ccdgpu_result_free.argtypes = [ctypes.POINTER(abi.Result)]
    L.ccdgpu_destroy.argtypes = [ctypes.c_void_p]
    ctx = ctypes.c_void_p()
    assert L.ccdgpu_init(0, ctypes.byref(ctx)) == 0
    out = {}
    for name in golden_util.names():
        if name == 'dense_daily':  # peek 96: past that build's 64 cap
            continue
        (d, s, q), params, ref = golden_util.load(name)
        p = abi.params_from_dict(params)
        import numpy as np
        d, s, q = (np.ascontiguousarray(x) for x in (d, s, q))
        res = abi.Result()
        rc = L.ccdgpu_detect_batch(ctx, ctypes.byref(p), q.shape[0], q.shape[1], d.ctypes.data, s.ctypes.data,
                                   q.ctypes.data, ctypes.byref(res))
        u = abi.unpack(res)
        L.ccdgpu_result_free(ctypes.byref(res))
        probs, mr = parity_util.compare(u, ref)
        out[name] = (rc, len(probs), u.segments.tobytes() + u.mask.tobytes())
    L.ccdgpu_destroy(ctx)
    return out


if __name__ == '__main__':
    lib_name = sys.argv[1]
    variants = sys.argv[2].split(',') if len(sys.argv) > 2 else ['w1', 'w2', 'w3', 'w4']
    base = run(lib_name, 'w3')
    rep = {'lib': lib_name}
    for v in variants:
        r = base if v == 'w3' else run(lib_name, v)
        rep[v] = {n: {'rc': r[n][0], 'golden_problems': r[n][1], 'identical_to_w3': r[n][2] == base[n][2]} for n in r}
    print(json.dumps(rep))
