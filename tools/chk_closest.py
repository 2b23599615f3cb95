"""Developer check: run golden vectors through a -DCCD_CHECK_CLOSEST build and report the first
closest-DOY comparison-rmse mismatch between the bucket path and the full selection scan."""
import os, sys, struct
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ['CCDGPU_LIBRARY'] = os.path.join(ROOT, 'lcmap-firebird_amd', 'lib', 'libccdgpu_chk.so')
sys.path.insert(0, os.path.join(ROOT, 'lcmap-firebird_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import ccdgpu
import golden_util
ctx = ccdgpu.Context(0)
for name in golden_util.names():
    (d, s, q), params, ref = golden_util.load(name)
    try:
        ctx.detect_batch(d, s, q, params=params)
    except Exception as e:
        print(name, 'error', e)
    dc = ctx.diag_counters()
    f = lambda x: struct.unpack('<d', struct.pack('<Q', x))[0]
    if dc[28]:
        print(name, 'MISMATCH nf', dc[28] - 1, 'K', dc[29] & 0xFFFF, 'less', (dc[29] >> 16) & 0xFFFF, 'T', dc[29] >> 32,
              'bucket', f(dc[30]), 'scan', f(dc[31]))
    else:
        print(name, 'ok')
