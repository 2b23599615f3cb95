#!/usr/bin/env python3
"""Static check for instructions stranded under a narrowed EXEC at an `if` join (developer tool).

LLVM's SILowerControlFlow (ROCm 7.2) drops the EXEC restore of a divergent `if` whose join block
falls straight into an enclosing region's restore ("redundant END_CF", option
-amdgpu-remove-redundant-endcf, default on).  The `if` is then lowered without saving EXEC
(`s_and_b64 sT, exec, cond; s_mov_b64 exec, sT`) and its join block keeps running with only the
`if`'s lanes enabled.  That is harmless while the join block is empty, but the register
allocator runs afterwards and does not model EXEC: a spill reload or copy it places in that join
block refills only the `if`'s lanes, and every other lane keeps a stale register (DESIGN.md §3,
the w4 divergence).

    python3 tools/endcf_check.py kernel.s [function-substring]

Reports, per function, every `if` lowered without an EXEC save whose join block holds an
instruction that writes a VGPR or reads/writes scratch before EXEC is restored.
"""
import re
import sys

NEUTRAL = re.compile(r'^(s_waitcnt|s_nop|s_barrier|s_branch|s_cbranch|s_setprio|s_sleep)')


def functions(path):
    funcs, cur = {}, None
    for raw in open(path):
        m = re.match(r'^([A-Za-z_][\w.$]*):', raw)
        if m and not m.group(1).startswith('.L'):
            cur = m.group(1)
            funcs[cur] = []
            continue
        if cur is not None:
            funcs[cur].append(raw.rstrip('\n'))
    return funcs


def instrs(body):
    """[(label or None, text)] with comments and directives dropped; labels as ('L', name)."""
    out = []
    for raw in body:
        s = raw.strip()
        m = re.match(r'^(\.LBB[\w_]+):', s)
        if m:
            out.append(('L', m.group(1)))
            continue
        t = s.split(';')[0].strip()
        if t and not t.startswith('.'):
            out.append(('I', t))
    return out


def check(name, body, verbose=True):
    ins = instrs(body)
    label_at = {t: i for i, (k, t) in enumerate(ins) if k == 'L'}
    found = 0
    narrowed = 0
    for i, (k, t) in enumerate(ins):
        if k != 'I':
            continue
        if re.match(r'^s_and_b64 exec, (exec, \S+|\S+, exec)$', t):
            unsaved_direct = True
        else:
            unsaved_direct = False
            m = re.match(r'^s_mov_b64 exec, (s\[\d+:\d+\])$', t)
            if not m:
                continue
            reg = m.group(1)
        # definition of the new mask: AND directly with exec (no saved copy) = no END_CF restore
        unsaved = unsaved_direct
        halves = ()
        if not unsaved_direct:
            lo, hi = [int(x) for x in reg[2:-1].split(':')]
            halves = (reg, 's%d' % lo, 's%d' % hi)
        for k2, t2 in ([] if unsaved_direct else reversed(ins[max(0, i - 2000):i])):
            if k2 == 'L':
                break  # definition in another block: not the lowering's own AND
            if k2 == 'I' and re.match(r'^[sv]_\w+ (%s),' % '|'.join(re.escape(h) for h in halves), t2):
                unsaved = bool(re.match(r'^s_and_b64 %s, (exec, \S+|\S+, exec)$' % re.escape(reg), t2))
                break
        if not unsaved:
            continue
        # the join: target of the s_cbranch_execz that follows
        join = None
        for k2, t2 in ins[i + 1:i + 4]:
            mm = re.match(r'^s_cbranch_execz (\.LBB[\w_]+)$', t2) if k2 == 'I' else None
            if mm:
                join = mm.group(1)
                break
        if join is None or join not in label_at:
            continue
        narrowed += 1
        bad = []
        # walk every path from the join until EXEC is written again (fall-through, branches)
        stack, seen = [label_at[join] + 1], set()
        while stack:
            pos = stack.pop()
            if pos in seen:
                continue
            seen.add(pos)
            while pos < len(ins):
                k2, t2 = ins[pos]
                pos += 1
                if k2 == 'L':
                    continue
                op = t2.split()[0]
                if re.match(r'^s_\w+ exec, ', t2) or op.startswith(('s_and_saveexec', 's_or_saveexec', 's_andn2_saveexec')):
                    break
                if op in ('s_endpgm', 's_setpc_b64'):
                    break
                mb = re.match(r'^s_(c?)branch\w* (\.LBB[\w_]+)$', t2)
                if mb:
                    if mb.group(2) in label_at:
                        stack.append(label_at[mb.group(2)] + 1)
                    if not mb.group(1):
                        break
                    continue
                if NEUTRAL.match(op):
                    continue
                writes_v = op.startswith(('v_', 'scratch_load', 'global_load', 'buffer_load', 'ds_read', 'flat_load')) and \
                    not op.startswith(('v_readlane', 'v_readfirstlane', 'v_cmp_')) and \
                    re.match(r'^\S+ v', t2) is not None
                if writes_v or op.startswith(('scratch_', 'buffer_store')):
                    bad.append(t2)
        if bad:
            found += 1
            if verbose:
                print('%s: if at "%s" -> join %s runs under the if\'s EXEC:' % (name[:48], t, join))
                for b in bad[:6]:
                    print('      ' + b)
    return narrowed, found


def main(path, only=None):
    total = 0
    for name, body in functions(path).items():
        if only and only not in name:
            continue
        narrowed, found = check(name, body)
        print('%s: %d ifs without an EXEC save, %d with VGPR/scratch work in their narrowed join' % (name[:60], narrowed, found))
        total += found
    return total


if __name__ == '__main__':
    sys.exit(1 if main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None) else 0)
