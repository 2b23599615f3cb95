"""Instruction mix of the detection kernel's loops that carry a given source-line range (developer
tool; reads the assembly tools/spill_map.py leaves in /tmp/spill_map/k.s).
Usage: python tools/loop_mix.py FIRST_LINE LAST_LINE [--kernel w3] [--print]"""
import collections
import re
import sys

lo, hi = int(sys.argv[1]), int(sys.argv[2])
kern = sys.argv[sys.argv.index('--kernel') + 1] if '--kernel' in sys.argv else 'w3'
name = {'w1': '_ZN12_GLOBAL__N_110ccd_detectEi', 'w2': '_ZN12_GLOBAL__N_113ccd_detect_w2Ei',
        'w3': '_ZN12_GLOBAL__N_113ccd_detect_w3Ei', 'w4': '_ZN12_GLOBAL__N_113ccd_detect_w4Ei'}[kern]
text = open('/tmp/spill_map/k.s').read()
s = text.index(name + ':')
lines = text[s:text.find('.Lfunc_end', s)].split('\n')
labels = {m.group(1): i for i, l in enumerate(lines) for m in [re.match(r'^(\.LBB\S+):', l)] if m}
loops = []
for i, l in enumerate(lines):
    m = re.search(r's_c?branch\w*\s+(\.LBB\S+)', l)
    if m and m.group(1) in labels and labels[m.group(1)] < i:
        loops.append((labels[m.group(1)], i))


def classify(op, ops):
    if op.startswith('v_'):
        if 'f64' in op:
            return 'valu_f64'
        if 'dpp' in op or 'row_' in ops or 'quad_perm' in ops:
            return 'valu_dpp'
        return 'valu_other'
    if op.startswith('s_nop'):
        return 's_nop'
    if op.startswith('s_waitcnt'):
        return 's_waitcnt'
    if op.startswith('s_'):
        return 'salu/branch'
    if op.startswith('ds_'):
        return 'lds'
    if op.startswith(('global_', 'buffer_', 'flat_')):
        return 'vmem'
    if op.startswith('scratch_'):
        return 'scratch'
    return 'other'


for a, b in loops:
    body = lines[a:b + 1]
    cur, inrange, total = None, 0, 0
    mix = collections.Counter()
    for x in body:
        mm = re.match(r'\s*\.loc\s+\d+\s+(\d+)', x)
        if mm:
            cur = int(mm.group(1))
            continue
        t = x.strip()
        if not t or t.startswith(('.', ';')) or t.endswith(':'):
            continue
        total += 1
        if cur is not None and lo <= cur <= hi:
            inrange += 1
        parts = t.split(None, 1)
        mix[classify(parts[0], parts[1] if len(parts) > 1 else '')] += 1
    inner = not any(c > a and d < b for c, d in loops)
    if total and inrange / total > 0.5 and inner:
        print('loop %d-%d: %d instructions, %.0f%% in lines %d-%d: %s' % (a, b, total, 100 * inrange / total, lo, hi, dict(mix)))
        if '--print' in sys.argv:
            print('\n'.join(x for x in body if x.strip() and not x.strip().startswith(('.loc', '.Ltmp', ';'))))
