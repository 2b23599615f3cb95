"""Developer tool (GPU box): golden-vector parity of one kernel library (CCDGPU_LIBRARY), one
line of problem counts per golden case.  Used to bisect a parity regression across builds."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'lcmap-firebird_amd'), os.path.join(ROOT, 'tests')]
import ccdgpu, golden_util, parity_util
ctx = ccdgpu.Context(0)
out = []
for name in golden_util.names():
    (d, s, q), params, ref = golden_util.load(name)
    got = ctx.detect_batch(d, s, q, params=params)
    probs, mr = parity_util.compare(got, ref)
    out.append('%s:%d' % (name, len(probs)))
print(os.path.basename(os.environ.get('CCDGPU_LIBRARY', 'default')), ' '.join(out), flush=True)
dc = ctx.diag_counters()
if dc[28]:
    import struct
    f = lambda u: struct.unpack('<d', struct.pack('<Q', u))[0]
    print('check tripped: tag %d  cnt %d m %d kk %d all %d  got %r ref %r' % (dc[28], dc[29] & 0xFFFF, (dc[29] >> 16) & 0xFFFF, (dc[29] >> 32) & 0xFFFF, dc[29] >> 48, f(dc[30]), f(dc[31])))
