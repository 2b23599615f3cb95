#!/usr/bin/env python3
"""Developer tool: static instruction counts per kernel source line from a -gline-tables-only
assembly (.loc of file 0 = the kernel source; the innermost kernel line of each inline chain).

    hipcc ... -gline-tables-only --cuda-device-only -S ccd_kernels.hip -o k.s
    python3 tools/isa_lines.py k.s ccd_detect_w3 FIRST LAST     # lines FIRST..LAST
"""
import re
import sys
from collections import Counter, defaultdict


def main(path, fn, first, last):
    body, on = [], False
    for ln in open(path):
        if re.match(r'^_Z\w*%s\w*:' % fn, ln):
            on = True
            continue
        if on and re.match(r'^_Z\w+:', ln):
            break
        if on:
            body.append(ln)
    cur = None
    cnt, ops = Counter(), defaultdict(Counter)
    for ln in body:
        m = re.match(r'\s+\.loc\s+(\d+)\s+(\d+)\s', ln)
        if m:
            if m.group(1) == '0':
                cur = int(m.group(2))
            else:  # a header line: keep the innermost kernel line of the chain
                k = re.findall(r'ccd_kernels\.hip:(\d+):', ln)
                cur = int(k[0]) if k else cur
            continue
        t = ln.strip()
        if not t or t.startswith(('.', ';')) or t.endswith(':') or cur is None:
            continue
        op = t.split()[0]
        cnt[cur] += 1
        ops[cur][op] += 1
    for line in range(first, last + 1):
        if cnt[line]:
            print('%5d %5d  %s' % (line, cnt[line], ' '.join('%s:%d' % kv for kv in ops[line].most_common(8))))
    print('total', sum(cnt[l] for l in range(first, last + 1)))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
