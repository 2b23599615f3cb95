"""Where the detection kernel's register spills sit (developer tool): compiles ccd_kernels.hip for
gfx950 with line tables, takes ccd_detect_w3 (or --kernel NAME), and lists every loop (backward
branch) that holds scratch spill loads/stores, with the source lines those spills carry and the
loop's nesting depth, innermost loops first.  Spills inside hot loops cost memory traffic and
latency on every iteration; spills at the top level cost almost nothing.
Usage: python tools/spill_map.py [--kernel w4] [--src path.hip]"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TMP = '/tmp/spill_map'
os.makedirs(TMP, exist_ok=True)
src = sys.argv[sys.argv.index('--src') + 1] if '--src' in sys.argv else os.path.join(ROOT, 'lcmap-firebird_amd', 'csrc', 'ccd_kernels.hip')
kern = sys.argv[sys.argv.index('--kernel') + 1] if '--kernel' in sys.argv else 'w3'
out = os.path.join(TMP, 'k.s')
if '--asm' in sys.argv:  # an existing -gline-tables-only assembly (e.g. built with the product's flags)
    out = sys.argv[sys.argv.index('--asm') + 1]
else:
  subprocess.check_call(['hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-ffp-contract=on', '-gline-tables-only',
                       '--cuda-device-only', '-S', '-I' + os.path.join(ROOT, 'include'), src, '-o', out],
                      stderr=subprocess.DEVNULL)
text = open(out).read()
name = {'w1': '_ZN12_GLOBAL__N_110ccd_detectEi', 'w2': '_ZN12_GLOBAL__N_113ccd_detect_w2Ei',
        'w3': '_ZN12_GLOBAL__N_113ccd_detect_w3Ei', 'w4': '_ZN12_GLOBAL__N_113ccd_detect_w4Ei'}[kern]
start = text.index(name + ':')
end = text.find('.Lfunc_end', start)
lines = text[start:end].split('\n')
labels = {m.group(1): i for i, l in enumerate(lines) for m in [re.match(r'^(\.LBB\S+):', l)] if m}
loops = []
for i, l in enumerate(lines):
    m = re.search(r's_c?branch\w*\s+(\.LBB\S+)', l)
    if m and m.group(1) in labels and labels[m.group(1)] < i:
        loops.append((labels[m.group(1)], i))
spill_pat = re.compile(r'scratch_(load|store)|buffer_(load|store)_dword\S*\s.*off(en|set).*s\[0:3\]')
cur = None
spills = []
for i, l in enumerate(lines):
    mm = re.match(r'\s*\.loc\s+\d+\s+(\d+)', l)
    if mm:
        cur = int(mm.group(1))
    if spill_pat.search(l):
        spills.append((i, cur, 'store' if 'store' in l else 'load'))
print('%s: %d spill instructions, %d loops' % (kern, len(spills), len(loops)))
rows = []
for a, b in loops:
    inside = [s for s in spills if a <= s[0] <= b]
    if not inside:
        continue
    depth = sum(1 for c, d in loops if c <= a and b <= d)
    inner = [s for s in inside if not any(c > a and d < b and c <= s[0] <= d for c, d in loops)]
    if not inner:
        continue
    locs = collections.Counter(s[1] for s in inner)
    rows.append((depth, b - a, len(inner), dict(sorted(locs.items()))))
for depth, ln, n, locs in sorted(rows, key=lambda r: (-r[0], -r[2])):
    print('depth %d  loop len %5d  spills %3d  source lines %s' % (depth, ln, n, locs))
top = [s for s in spills if not any(a <= s[0] <= b for a, b in loops)]
print('outside any loop: %d' % len(top))
