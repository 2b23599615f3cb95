"""Parity soak on the GPU box (developer tool): whole tile chips through the HIP path (one ragged
batch per config, ccdgpu_stage_chips) against the C restatement oracle on the same inputs, with
the test suite's parity bar (tests/parity_util.py: every integer / index output exact, floats
within 1e-6 relative).  Chips are spread over the synthetic tile so both cadences (base 1421 obs,
sidelap 2121 obs) are covered.  Prints one JSON summary.
Usage: python tools/parity_soak.py [C3 chips] [C5 chips] [oracle threads] [C2 chips] [C4 chips]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ('lcmap-firebird_amd', 'oracle', 'tests'):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np  # noqa: E402
import ccdgpu  # noqa: E402
import oracle_ctypes  # noqa: E402
import parity_util  # noqa: E402
from ccdgpu import synth  # noqa: E402


def soak(which, n_chips, threads, ctx):
    cfg = synth.config(which)
    ids = [int(round(i * 2499.0 / max(1, n_chips - 1))) for i in range(n_chips)]
    out = {'config': which, 'chips': ids, 'pixels': 0, 'segments': 0, 'n_obs': {}, 'mismatched_pixels': 0,
           'problems': [], 'max_rel': 0.0, 'gpu_s': 0.0, 'oracle_s': 0.0}
    for c in ids:
        d, s, q = synth.chip(cfg, c, 0, 10000)
        t0 = time.time()
        got = ctx.detect_batch(d, s, q)
        t1 = time.time()
        rc, ref = oracle_ctypes.detect_batch(d, s, q, threads=threads)
        t2 = time.time()
        assert rc == 0, rc
        problems, max_rel = parity_util.compare(got, ref, max_report=10 ** 9)
        bad = {int(p.split()[1]) for p in problems if p.startswith('px ')}
        out['pixels'] += q.shape[0]
        out['segments'] += int(got.segments.shape[0])
        out['n_obs'][str(d.shape[0])] = out['n_obs'].get(str(d.shape[0]), 0) + 1
        out['mismatched_pixels'] += len(bad) + (0 if not problems or bad else 1)
        out['problems'] += ['chip %d: %s' % (c, p) for p in problems[:5]]
        out['max_rel'] = max(out['max_rel'], max_rel)
        out['gpu_s'] += t1 - t0
        out['oracle_s'] += t2 - t1
        print('config %d chip %d n_obs %d: %d problems, max rel %.2e (gpu %.2fs, oracle %.1fs)' % (
            which, c, d.shape[0], len(problems), max_rel, t1 - t0, t2 - t1), file=sys.stderr, flush=True)
    return out


def main():
    n3 = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    n5 = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    threads = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    n2 = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    n4 = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    ctx = ccdgpu.Context(0)
    res = {'tool': 'tools/parity_soak.py', 'library': ccdgpu.LIB_PATH, 'bar': 'tests/parity_util.py (ints exact, '
           'floats 1e-6 rel)', 'oracle': 'oracle/ccd_oracle.c (C restatement), %d threads' % threads,
           'runs': [soak(w, n, threads, ctx) for w, n in ((3, n3), (5, n5), (2, n2), (4, n4)) if n]}
    ctx.close()
    res['pixels'] = sum(r['pixels'] for r in res['runs'])
    res['mismatched_pixels'] = sum(r['mismatched_pixels'] for r in res['runs'])
    print(json.dumps(res, indent=1))
    return 0 if res['mismatched_pixels'] == 0 else 1


if __name__ == '__main__':
    sys.exit(main())
