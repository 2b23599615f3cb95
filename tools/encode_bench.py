#!/usr/bin/env python3
"""Host encoder throughput (ccdgpu_encode_chips) on this machine's CPU: raw input GB/s of the
'unread' and 'lossless' settings at 1 and 3 threads over distinct synthetic tile chips (C3
cadences, 10,000 pixels), beside a plain copy of the same arrays into the same kind of buffer.

usage: encode_bench.py [n_chips] [reps]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'lcmap-firebird_amd'))
import ccdgpu  # noqa: E402
from ccdgpu import synth  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    cfg = synth.config(3)
    t = time.perf_counter()
    chips = [synth.chip(cfg, c, 0, 10000) for c in range(n)]
    print('generated %d chips in %.1f s' % (n, time.perf_counter() - t), flush=True)
    raw = sum(s.nbytes + q.nbytes for _, s, q in chips)
    e = ccdgpu.EncodedBatch([q.shape[0] for _, _, q in chips], [d.shape[0] for d, _, _ in chips], pinned=False)
    dst = np.empty(raw, dtype=np.uint8)
    out = {'raw_bytes': raw, 'vector_path': ccdgpu.encode_vector_path()}
    for threads in (1, 3):
        for name, (drop, strict) in (('unread', ccdgpu.unread_drop_bits(None)), ('lossless', (1, 1))):
            best = 1e9
            for _ in range(reps):
                t = time.perf_counter()
                nb = e.fill(chips, threads=threads, drop_bits=drop, strict_bits=strict)
                best = min(best, time.perf_counter() - t)
            out['%s_t%d_gbs' % (name, threads)] = round(raw / best / 1e9, 2)
            out['%s_sent_frac' % name] = round(nb / raw, 3)
        best = 1e9
        for _ in range(reps):
            t = time.perf_counter()
            pos = 0
            for _, s, q in chips:  # (single-threaded numpy copies, for scale)
                for a in (s, q):
                    dst[pos:pos + a.nbytes] = a.reshape(-1).view(np.uint8)
                    pos += a.nbytes
            best = min(best, time.perf_counter() - t)
        out['copy_t1_gbs'] = round(raw / best / 1e9, 2)
    print(out)


if __name__ == '__main__':
    main()
