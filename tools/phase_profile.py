"""Per-phase cycle breakdown of the detection kernel (diagnostic build lib/libccdgpu_diag.so).
Run on the GPU box:  python tools/phase_profile.py [config] [chips]"""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault('CCDGPU_LIBRARY', os.path.join(ROOT, 'lcmap-firebird_amd', 'lib', 'exp', os.environ.get('CCD_DIAG_LIB', 'libccdgpu_diag.so')))
sys.path.insert(0, os.path.join(ROOT, 'lcmap-firebird_amd'))
import numpy as np
import ccdgpu
from ccdgpu import synth
which = int(sys.argv[1]) if len(sys.argv) > 1 else 3
chips = int(sys.argv[2]) if len(sys.argv) > 2 else 2
cfg = synth.config(which)
ids = [c for c in range(64) if synth.dates(cfg, c).shape[0] == synth.dates(cfg, 0).shape[0]][:chips]
data = [synth.chip(cfg, c, 0, 10000) for c in ids]
ctx = ccdgpu.Context(0)
ctx.stage(np.stack([d[0] for d in data]), np.stack([d[1] for d in data]), np.stack([d[2] for d in data]))
ctx.run()
st, dc = ctx.stats(), ctx.diag_counters()
names = ['pixel total', 'QA/filter/compact', 'variogram+peek', 'tmask', 'lasso gram', 'lasso cd',
         'lasso rmse', 'lf batch', 'single-step peek eval', 'outlier compaction', 'stability', 'medians+emit',
         'closest bucket build', 'batch: ring residuals', 'batch: closest-doy (lane)', 'batch: magnitudes']
counts = ['batched steps', 'batches', 'single-step peek evals', 'fit calls']
tot = dc[8] or 1
out = {'config': which, 'chips': chips, 'detect_ms': st['detect_ms'], 'fits': dc[0], 'sweeps': dc[1],
       'sweeps_per_fit': dc[1] / max(1, dc[0] / 7)}
for i, n in enumerate(names):
    out[n] = dc[8 + i] / tot
for i, n in enumerate(counts):
    out[n] = dc[8 + 16 + i]
for i, n in enumerate(['spec early fits (CD)', 'closest: search', 'closest: run sum', 'closest: ties']):
    out[n] = dc[8 + 20 + i] / tot
# default kernel (bucket records + bounded magnitudes): slot 21 counts the steps whose comparison
# rmse was computed (coop_comp); comp_lane's sub-phase timers 21-23 belong to the CCD_BUCKET_R2 build
out['steps with comparison rmse (coop_comp)'] = dc[8 + 21]
for i, n in enumerate(['batches ne<=16', 'batches ne<=32', 'batch valid lanes', 'batches without terminal step',
                       'wave fits at max_iter', 'wave sweeps (single fits)', 'wave sweeps in max_iter fits',
                       'compaction rows scanned']):
    out[n] = dc[8 + 24 + i]
for i, n in enumerate(['init tmask calls', 'init fits', 'lf batched refits', 'spec calls', 'spec windows computed',
                       'spec windows installed', 'spec wave sweeps', 'spec lane sweeps']):
    out[n] = dc[8 + 32 + i]
if os.environ.get('CCD_DIAG_LIB', '').endswith('cdcyc.so'):
    # CCD_CD_CYCLES build: slots 24-27 = band groups that ran max_iter sweeps, those of them whose
    # sweep state repeated (a cycle), sum of their detection sweeps, sum of their periods
    for i, n in enumerate(['batches ne<=16', 'batches ne<=32', 'batch valid lanes', 'batches without terminal step']):
        out.pop(n, None)
    g, c, it, per = dc[8 + 24], dc[8 + 25], dc[8 + 26], dc[8 + 27]
    out['cd groups at max_iter'] = g
    out['cd groups at max_iter that cycled'] = c
    out['mean detection sweep'] = it / c if c else None
    out['mean period'] = per / c if c else None
if os.environ.get('CCD_DIAG_LIB', '').endswith('cdchk.so'):
    # CCD_CD_CHKSTAT build: slots 24-27 = coordinate-descent wave sweeps (cd_sweep), those that take
    # the duality-gap test, those whose live band groups sit in one half of their 16-lane rows,
    # those whose float pre-check of the stopping ratio was ambiguous
    for i, n in enumerate(['batches ne<=16', 'batches ne<=32', 'batch valid lanes', 'batches without terminal step']):
        out.pop(n, None)
    sw = dc[8 + 24] or 1
    out['cd wave sweeps'] = dc[8 + 24]
    out['cd sweeps with gap test'] = dc[8 + 25] / sw
    out['cd sweeps with live groups in one row half'] = dc[8 + 26] / sw
    out['cd sweeps with ambiguous ratio pre-check'] = dc[8 + 27] / sw
out['pixels'] = chips * 10000
out['cycles_per_pixel'] = tot / out['pixels']
print(json.dumps(out, indent=1))
