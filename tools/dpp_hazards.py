#!/usr/bin/env python3
"""Static check of the gfx950 software wait-state hazards that matter to the detection kernel
(developer tool; `make -C lcmap-firebird_amd isa-check` runs it over lib/ccd_kernels.s).

The compiler pads the hazards of instructions it generates, but an inline-asm statement is
opaque to its hazard recognizer: a hazard whose producer or consumer sits inside an `asm`
string is padded only if the string pads it.  Rules checked (CDNA3/CDNA4 ISA, "manually
inserted wait states"; the accumulator rule measured on gfx950 with tools/probe/dpp64.hip):

  dpp-src    VALU writes a VGPR       -> DPP op reads it (source or v_fmac accumulator)   2
  exec-dpp   VALU writes EXEC (cmpx)  -> any DPP op                                       5
  sgpr-lane  VALU writes an SGPR      -> v_readlane / v_writelane lane select reads it     4
  sgpr-vmem  VALU writes an SGPR      -> VMEM / scratch / global instruction reads it      5
  vcc-fmas   VALU writes VCC          -> v_div_fmas                                        4
  trans-use  VALU transcendental      -> non-transcendental VALU reads its result          1
  vgpr-lane  VALU writes a VGPR       -> v_readlane / v_readfirstlane reads it             1

    python3 tools/dpp_hazards.py kernel.s|kernel.dis [--all]

Walks each function linearly (a conservative approximation across branches: a label resets
nothing).  By default only hazards with an inline-asm instruction on either side are reported
(the compiler's own code is its hazard recognizer's job); --all reports every one.
"""
import re
import sys

DPP_RE = re.compile(r'(_dpp\b|row_newbcast|quad_perm|row_shr|row_shl|row_ror|row_bcast|row_mirror|row_half_mirror|wave_shr|wave_shl|wave_ror|wave_rol)')
VREG_RE = re.compile(r'\bv(\d+)\b|\bv\[(\d+):(\d+)\]')
SREG_RE = re.compile(r'\bs(\d+)\b|\bs\[(\d+):(\d+)\]|\b(vcc)\b|\b(exec)\b')
TRANS = ('v_exp_', 'v_log_', 'v_rcp_', 'v_rsq_', 'v_sqrt_', 'v_sin_', 'v_cos_', 'v_rcp_iflag')
VMEM = ('global_', 'scratch_', 'buffer_', 'flat_')
SDST_VALU = ('v_readlane', 'v_readfirstlane', 'v_cmp_', 'v_cmpx_', 'v_div_scale', 'v_add_co', 'v_sub_co',
             'v_subrev_co', 'v_addc_co', 'v_subb_co', 'v_mad_u64', 'v_mad_i64')


def vregs(text):
    out = set()
    for m in VREG_RE.finditer(text):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def sregs(text):
    out = set()
    for m in SREG_RE.finditer(text):
        if m.group(1) is not None:
            out.add('s%s' % m.group(1))
        elif m.group(2) is not None:
            out.update('s%d' % i for i in range(int(m.group(2)), int(m.group(3)) + 1))
        elif m.group(4):
            out.update(('vcc', 's106', 's107'))
        else:
            out.add('exec')
    return out


def fields(ops):
    return [f.strip() for f in ops.split(',')] if ops else []


def classify(op, ops):
    """(vgpr dsts, sgpr dsts, vgpr srcs, sgpr srcs) of one instruction."""
    f = fields(ops)
    vd, sd, vs, ss = set(), set(), set(), set()
    if op.startswith('v_'):
        if op.startswith(('v_readlane', 'v_readfirstlane')):
            sd = sregs(f[0]) if f else set()
        elif op.startswith('v_cmpx'):
            sd = {'exec'}
            if f and not f[0].startswith('v'):
                sd |= sregs(f[0])
        elif op.startswith('v_cmp'):
            sd = sregs(f[0]) if f and (f[0].startswith('s') or f[0] == 'vcc') else {'vcc', 's106', 's107'}
        else:
            vd = vregs(f[0]) if f else set()
            if op.startswith(SDST_VALU) and len(f) > 1 and (f[1].startswith('s') or f[1] == 'vcc'):
                sd = sregs(f[1])
        srcs = f[1:]
        if op.startswith(('v_fmac', 'v_mac')):
            srcs = f
        for x in srcs:
            tok = x.split(' ')[0]
            vs |= vregs(tok)
            ss |= sregs(tok)
    else:
        for x in f:
            tok = x.split(' ')[0]
            vs |= vregs(tok)
            ss |= sregs(tok)
    return vd, sd, vs, ss


def parse(line):
    line = line.split('//')[0].split(';')[0].strip()
    if not line or line.endswith(':') or line.startswith(('Disassembly', '.')):
        return None
    parts = line.split(None, 1)
    return parts[0], parts[1] if len(parts) > 1 else ''


def main(path, all_hazards=False):
    hist = []  # (wait states, op, vdst, sdst, is_trans, in_asm, text)
    func = '?'
    found = 0
    in_asm = False
    for raw in open(path):
        s = raw.strip()
        if s.endswith('>:') or re.match(r'^_Z\w+:', s):
            func = s
            hist = []
            continue
        if s.startswith(';;#ASMSTART'):
            in_asm = True
            continue
        if s.startswith(';;#ASMEND'):
            in_asm = False
            continue
        p = parse(raw)
        if p is None:
            continue
        op, ops = p
        vd, sd, vs, ss = classify(op, ops)
        is_valu = op.startswith('v_')
        dpp = is_valu and DPP_RE.search(op + ' ' + ops) is not None
        text = s.split(';')[0].split('//')[0]
        checks = []  # (rule, need, predicate on a history entry)
        if dpp:
            checks.append(('dpp-src', 2, lambda h, vs=vs: h[1].startswith('v_') and h[2] & vs))
            checks.append(('exec-dpp', 5, lambda h: h[1].startswith('v_') and 'exec' in h[3]))
        if op.startswith(('v_readlane', 'v_writelane')):
            f = fields(ops)
            lane_sel = sregs(f[-1].split(' ')[0]) if f else set()
            checks.append(('sgpr-lane', 4, lambda h, ls=lane_sel: h[1].startswith('v_') and h[3] & ls))
        if op.startswith(('v_readlane', 'v_readfirstlane')):
            checks.append(('vgpr-lane', 1, lambda h, vs=vs: h[1].startswith('v_') and h[2] & vs))
        if op.startswith(VMEM):
            checks.append(('sgpr-vmem', 5, lambda h, ss=ss: h[1].startswith('v_') and h[3] & ss))
        if op.startswith('v_div_fmas'):
            checks.append(('vcc-fmas', 4, lambda h: h[1].startswith('v_') and 'vcc' in h[3]))
        if is_valu and not op.startswith(TRANS):
            checks.append(('trans-use', 1, lambda h, vs=vs: h[4] and h[2] & vs))
        for rule, need, pred in checks:
            ws = 0
            for h in reversed(hist):
                if ws >= need:
                    break
                if pred(h):
                    if all_hazards or in_asm or h[5]:
                        found += 1
                        print('%s\n    [%s] %s\n    after %s (%d of %d wait states)' % (func[:60], rule, text, h[6], ws, need))
                    break
                ws += h[0]
        w = int(ops.strip() or '0', 0) + 1 if op == 's_nop' else 1
        hist.append((w, op, vd, sd, is_valu and op.startswith(TRANS), in_asm, text))
        if len(hist) > 12:
            hist.pop(0)
    print('%d potential wait-state hazards%s' % (found, '' if all_hazards else ' involving inline asm'))
    return found


if __name__ == '__main__':
    sys.exit(1 if main(sys.argv[1], '--all' in sys.argv[2:]) else 0)
