#!/usr/bin/env python3
"""Static check of the VALU-write -> DPP-read hazard in a gfx950 disassembly (developer tool).

CDNA needs 2 wait states between a VALU instruction that writes a VGPR and a DPP instruction
that reads it (the DPP source, and -- measured on gfx950 with tools/probe/dpp64.hip -- the
accumulator of v_fmac_f64_dpp).  The compiler inserts the s_nop for instructions it knows, but
inline asm is opaque to its hazard recognizer, so a DPP op right after an inline-asm VALU write
(or an inline-asm DPP op right after a compiler VALU write) can read a stale value.

    llvm-objdump -d --no-show-raw-insn k.out > k.dis; python3 tools/dpp_hazards.py k.dis

Walks each function linearly (a conservative approximation across branches: a label resets
nothing, so a hazard across a taken branch edge is reported as if fall-through) and reports every
DPP instruction with a VALU write to one of its VGPR sources fewer than 2 wait states before it.
"""
import re
import sys

DPP_RE = re.compile(r'(_dpp\b|row_newbcast|quad_perm|row_shr|row_shl|row_ror|row_bcast|row_mirror|row_half_mirror|wave_shr|wave_shl|wave_ror|wave_rol)')
REG_RE = re.compile(r'\bv(\d+)\b|\bv\[(\d+):(\d+)\]')


def regs(text):
    out = set()
    for m in REG_RE.finditer(text):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def parse(line):
    line = line.split('//')[0].strip()
    if not line or line.endswith(':') or line.startswith(('Disassembly', ';')):
        return None
    parts = line.split(None, 1)
    op = parts[0]
    ops = parts[1] if len(parts) > 1 else ''
    return op, ops


def dest_vgprs(op, ops):
    """VGPRs written by a VALU instruction (first operand when it is a VGPR)."""
    if not op.startswith('v_'):
        return set()
    if op.startswith(('v_readlane', 'v_readfirstlane', 'v_cmp')) and not op.startswith('v_cmpx'):
        return set()
    first = ops.split(',')[0]
    return regs(first)


def src_vgprs(op, ops):
    fields = [f.strip() for f in ops.split(',')]
    srcs = set()
    for f in fields[1:]:
        srcs |= regs(f.split(' ')[0])
    if op.startswith(('v_fmac', 'v_mac')):
        srcs |= regs(fields[0])  # accumulator
    return srcs


def main(path):
    hist = []  # (wait_states_of_instr, dest_vgprs, text)
    func = '?'
    found = 0
    for raw in open(path):
        if raw.rstrip().endswith('>:'):
            func = raw.strip()
            hist = []
            continue
        p = parse(raw)
        if p is None:
            continue
        op, ops = p
        if DPP_RE.search(op + ' ' + ops) and op.startswith('v_'):
            need = src_vgprs(op, ops)
            ws = 0
            for w, dst, txt in reversed(hist):
                if ws >= 2:
                    break
                if dst & need:
                    found += 1
                    print('%s\n    %s\n    after %s (%d wait states)' % (func[:60], raw.strip().split('//')[0], txt, ws))
                    break
                ws += w
        if op == 's_nop':
            w = int(ops.strip() or '0', 0) + 1
        else:
            w = 1
        hist.append((w, dest_vgprs(op, ops), raw.strip().split('//')[0]))
        if len(hist) > 8:
            hist.pop(0)
    print('%d potential VALU->DPP hazards' % found)
    return found


if __name__ == '__main__':
    sys.exit(1 if main(sys.argv[1]) else 0)
