#!/usr/bin/env python3
"""Static check: is SCC live across an inline-asm block that writes it? (developer tool)

hipcc treats an `asm` statement as opaque: unless the statement lists "scc" among its clobbers,
the register allocator and scheduler assume SCC survives it.  An asm block that writes SCC
(s_and_saveexec_b64, s_and_b64, s_cmp, ...) between a compiler SCC definition and a compiler
SCC reader (s_cbranch_scc*, s_cselect_*, s_addc/s_subb, s_cmov*) silently changes that
reader's input.  Whether the compiler happens to keep SCC live across the statement depends
on scheduling and register allocation, i.e. on the register budget of the build.

    python3 tools/asm_scc_live.py kernel.s [function-substring]

Walks each function of a -save-temps .s linearly and reports every asm block that writes SCC
while a compiler-defined SCC is read after it before being redefined.
"""
import re
import sys

SCC_READ = re.compile(r'^(s_cbranch_scc[01]|s_cselect_b(32|64)|s_addc_u32|s_subb_u32|s_cmovk_i32|s_cmov_b(32|64))$')
SCC_WRITE_PREFIX = ('s_cmp', 's_add_', 's_sub_', 's_addc', 's_subb', 's_and_', 's_or_', 's_xor_', 's_andn2', 's_orn2',
                    's_nand', 's_nor', 's_xnor', 's_lshl', 's_lshr', 's_ashr', 's_bfe', 's_min_', 's_max_', 's_not_',
                    's_bcnt', 's_abs', 's_addk', 's_bitcmp', 's_absdiff', 's_and_saveexec', 's_or_saveexec',
                    's_andn2_saveexec', 's_quadmask', 's_wqm')


def writes_scc(op):
    return op.startswith(SCC_WRITE_PREFIX)


def main(path, only=None):
    func = None
    lines = []
    funcs = {}
    for raw in open(path):
        m = re.match(r'^([A-Za-z_][\w.$]*):', raw)
        if m and not raw.startswith('.') and not m.group(1).startswith('.L'):
            func = m.group(1)
            funcs[func] = []
            continue
        if func is not None:
            funcs[func].append(raw.rstrip('\n'))
    bad = 0
    for f, body in funcs.items():
        if only and only not in f:
            continue
        # instructions: (kind, op, text); kind 'asm' for a whole asm block
        ins = []
        i = 0
        while i < len(body):
            s = body[i].strip()
            if s.startswith(';;#ASMSTART'):
                blk = []
                i += 1
                while i < len(body) and not body[i].strip().startswith(';;#ASMEND'):
                    t = body[i].split(';')[0].strip()
                    if t:
                        blk.append(t)
                    i += 1
                ins.append(('asm', blk, i))
            else:
                t = s.split(';')[0].strip()
                if t and not t.startswith('.') and not t.endswith(':'):
                    ins.append(('ins', t, i))
            i += 1
        for n, (kind, blk, ln) in enumerate(ins):
            if kind != 'asm' or not any(writes_scc(x.split()[0]) for x in blk):
                continue
            # forward: first SCC reader or writer after the block
            for kind2, t, ln2 in ins[n + 1:]:
                if kind2 == 'asm':
                    if any(writes_scc(x.split()[0]) for x in t):
                        break
                    continue
                op = t.split()[0]
                if SCC_READ.match(op):
                    # compiler reads SCC the asm block overwrote: was it defined by compiler code before?
                    bad += 1
                    print('%s: asm block ending at line %d (%s) is followed by SCC reader at line %d: %s'
                          % (f[:50], ln, ' ; '.join(blk), ln2, t))
                    break
                if writes_scc(op):
                    break
    print('%d asm blocks clobbering a live SCC' % bad)
    return bad


if __name__ == '__main__':
    sys.exit(1 if main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None) else 0)
