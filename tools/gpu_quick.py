"""Quick GPU-vs-oracle parity + timing probe (developer tool; runs on the GPU box)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'lcmap-firebird_amd'), os.path.join(ROOT, 'oracle'), os.path.join(ROOT, 'tests')]
import numpy as np
import ccdgpu
from ccdgpu import synth
import oracle_ctypes, parity_util

npix = int(sys.argv[1]) if len(sys.argv) > 1 else 64
ctx = ccdgpu.Context(0)
print('version', ccdgpu.version(), flush=True)
for which in (2, 4, 5):
    cfg = synth.config(which)
    d, s, q = synth.chip(cfg, 11, 0, npix)
    t = time.time(); u = ctx.detect_batch(d, s, q); tg = time.time() - t
    t = time.time(); rc, r = oracle_ctypes.detect_batch(d, s, q, threads=16); to = time.time() - t
    probs, mr = parity_util.compare(u, r)
    print('config %d npix %d: gpu %.3fs (kernel %.3fs) oracle %.3fs segs %d/%d problems %d maxrel %.2e' % (
        which, npix, tg, u.seconds_kernel, to, len(u.segments), len(r.segments), len(probs), mr), flush=True)
    for p in probs[:10]:
        print('   ', p)
    print('   stats', ctx.stats(), flush=True)
