"""ISA loop scan of the detection kernel (developer tool): for every loop of ccd_detect_w3, the
global loads and `s_waitcnt vmcnt(0)` waits it holds and the source lines of its loads.  A loop
with as many waits as loads consumes each load before issuing the next (serialised latency).
Usage: python tools/isa_loops.py [--lds]   (compiles with -gline-tables-only into /tmp/isa_loops)"""
import collections, os, re, subprocess, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TMP = '/tmp/isa_loops'
os.makedirs(TMP, exist_ok=True)
subprocess.check_call(['hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-gline-tables-only',
                       '-I' + os.path.join(ROOT, 'include'), '-c',
                       os.path.join(ROOT, 'lcmap-firebird_amd', 'csrc', 'ccd_kernels.hip'), '-o', 'k.o', '-save-temps'],
                      cwd=TMP, stderr=subprocess.DEVNULL)
asm = [f for f in os.listdir(TMP) if f.endswith('gfx950.s')][0]
text = open(os.path.join(TMP, asm)).read()
start = text.index('_ZN12_GLOBAL__N_113ccd_detect_w3Ev:')
end = text.find('_ZN12_GLOBAL__N_113ccd_detect_w4Ev:', start)
lines = text[start:end if end > 0 else None].split('\n')
lds = '--lds' in sys.argv
load_pat, wait_pat = ('ds_read', r'lgkmcnt\(0\)') if lds else ('global_load', r'vmcnt\(0\)')
labels = {m.group(1): i for i, l in enumerate(lines) for m in [re.match(r'^(\.LBB\S+):', l)] if m}
seen = set()
for i, l in enumerate(lines):
    m = re.search(r's_c?branch\w*\s+(\.LBB\S+)', l)
    if not (m and m.group(1) in labels and labels[m.group(1)] < i):
        continue
    body = lines[labels[m.group(1)]:i + 1]
    locs, cur = collections.Counter(), None
    for x in body:
        mm = re.match(r'\s*\.loc\s+\d+\s+(\d+)', x)
        if mm:
            cur = int(mm.group(1))
        if load_pat in x and cur:
            locs[cur] += 1
    if not locs or tuple(sorted(locs)) in seen:
        continue
    seen.add(tuple(sorted(locs)))
    nw = sum(1 for x in body if re.search(r's_waitcnt.*' + wait_pat, x))
    print('len %5d loads %3d waits %3d  source lines %s' % (len(body), sum(locs.values()), nw, dict(sorted(locs.items()))))
