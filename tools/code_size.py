"""Code size of the detection kernel by source function (developer tool): instruction counts of
the ccd_detect_w3 body (assembly from tools/spill_map.py, /tmp/spill_map/k.s) attributed through
the line table to the enclosing function of ccd_kernels.hip.  The kernel is one inlined body
several hundred KB long, far past the 64 KB instruction cache a CU pair shares.
Usage: python tools/code_size.py [--kernel w3]"""
import collections
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, 'lcmap-firebird_amd', 'csrc', 'ccd_kernels.hip')).read().split('\n')
kern = sys.argv[sys.argv.index('--kernel') + 1] if '--kernel' in sys.argv else 'w3'
name = {'w2': '_ZN12_GLOBAL__N_113ccd_detect_w2Ei', 'w3': '_ZN12_GLOBAL__N_113ccd_detect_w3Ei',
        'w4': '_ZN12_GLOBAL__N_113ccd_detect_w4Ei'}[kern]
# enclosing function of each source line: the last definition line at column 0 above it
fn_of, cur = {}, '?'
for i, l in enumerate(src, 1):
    m = re.match(r'^(?:template <[^>]*>\s*)?(?:__device__|__global__|static|extern)[^(]*?(\w+)\s*\(', l)
    if m and not l.rstrip().endswith(';'):
        cur = m.group(1)
    fn_of[i] = cur
text = open('/tmp/spill_map/k.s').read()
s = text.index(name + ':')
body = text[s:text.find('.Lfunc_end', s)].split('\n')
cnt, file_main, line = collections.Counter(), None, 0
files = {}
for x in text.split('\n'):
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', x)
    if m:
        files[m.group(1)] = (m.group(3) or m.group(2))
cur_file = None
for x in body:
    m = re.match(r'\s*\.loc\s+(\d+)\s+(\d+)', x)
    if m:
        cur_file, line = files.get(m.group(1), ''), int(m.group(2))
        continue
    t = x.strip()
    if not t or t.startswith(('.', ';')) or t.endswith(':'):
        continue
    key = fn_of.get(line, '?') if cur_file and cur_file.endswith('ccd_kernels.hip') else os.path.basename(cur_file or '?')
    cnt[key] += 1
tot = sum(cnt.values())
print('%s: %d instructions' % (kern, tot))
for k, v in cnt.most_common(30):
    print('%7d %5.1f%%  %s' % (v, 100.0 * v / tot, k))
