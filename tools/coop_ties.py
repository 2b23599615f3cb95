"""How often the exact comparison rmse (coop_comp) met more tied entries than the 24 need and a
selection of more entries than a wave (E > 64), on a golden vector -- diagnostic build's counters
(slots 21-23).  Run on the GPU box with CCDGPU_LIBRARY pointing at a diagnostic build:
    CCDGPU_LIBRARY=.../libccdgpu_diag.so python tools/coop_ties.py tie_cycles tie_cycles_stable"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'lcmap-firebird_amd'), os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'oracle')]
import ccdgpu  # noqa: E402
import golden_util  # noqa: E402
import parity_util  # noqa: E402

ctx = ccdgpu.Context(0)
out = {}
for name in sys.argv[1:]:
    (d, s, q), params, ref = golden_util.load(name)
    got = ctx.detect_batch(d, s, q, params=params)
    dc = ctx.diag_counters()
    problems, max_rel = parity_util.compare(got, ref)
    out[name] = {'library': os.path.basename(ccdgpu.LIB_PATH), 'pixels': int(q.shape[0]), 'obs': int(d.shape[0]),
                 'coop_comp_steps': dc[8 + 21], 'selections_over_64_entries': dc[8 + 22],
                 'ties_past_need': dc[8 + 23], 'parity_problems': len(problems), 'max_rel': max_rel}
print(json.dumps(out, indent=1))
