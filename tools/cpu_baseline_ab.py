#!/usr/bin/env python3
"""CPU-baseline sampling A/B (developer tool, GPU box host): the C restatement oracle on the
bench's resident batch, sampled as rounds 1-5 did (the first ~17k pixels of the chips sharing
chip 0's base-cadence dates) and as round 6 does (>= 2 x 10^4 pixels in the tile's cadence mix,
strided over each chip), back to back on the same host, plus the round-6 sampler restricted to the
base cadence -- which part of the round-6 baseline's rate is the sample and which the host."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'lcmap-firebird_amd'), os.path.join(ROOT, 'oracle')]
import numpy as np  # noqa: E402
import bench  # noqa: E402
import oracle_ctypes  # noqa: E402
from ccdgpu import synth  # noqa: E402


def timed(dates, S, Q, thr):
    t = time.perf_counter()
    oracle_ctypes.detect_batch(dates, S, Q, threads=thr)
    return time.perf_counter() - t


def main():
    cfg = synth.config(3)
    ids = bench.chip_ids(0, 64, 1, lambda c: bench.synth_nobs(cfg, c))
    t = time.perf_counter()
    batch = bench.build_batch(cfg, ids)
    print('batch built in %.1f s' % (time.perf_counter() - t), flush=True)
    thr, info = bench.host_cpus()
    d0 = batch.chip(0)[0]
    same = [c for c in range(batch.n_chips) if np.array_equal(batch.chip(c)[0], d0)]
    out = {'threads': thr, 'cpu': info}
    # rounds 1-5: the first n pixels of the chips sharing chip 0's dates (chip 0's 10^4, then the next)
    for n in (17000,):
        S = np.ascontiguousarray(np.concatenate([batch.chip(c)[1] for c in same[:2]], axis=1)[:, :n])
        Q = np.ascontiguousarray(np.concatenate([batch.chip(c)[2] for c in same[:2]], axis=0)[:n])
        timed(d0, S[:, :512], Q[:512], thr)
        el = timed(d0, S, Q, thr)
        out['first_%d_base_cadence' % n] = round(n / el, 1)
        print('first', n, round(n / el, 1), flush=True)
    # round 6, restricted to the base cadence: 392 pixels strided over each of 33 chips
    per = 392
    S = np.ascontiguousarray(np.concatenate([batch.chip(c)[1][:, np.linspace(0, 9999, per).astype(np.int64)] for c in same], axis=1))
    Q = np.ascontiguousarray(np.concatenate([batch.chip(c)[2][np.linspace(0, 9999, per).astype(np.int64)] for c in same], axis=0))
    el = timed(d0, S, Q, thr)
    out['strided_%d_base_cadence' % S.shape[1]] = round(S.shape[1] / el, 1)
    print('strided', S.shape[1], round(S.shape[1] / el, 1), flush=True)
    # the first 392 pixels of each of the 33 chips
    S = np.ascontiguousarray(np.concatenate([batch.chip(c)[1][:, :per] for c in same], axis=1))
    Q = np.ascontiguousarray(np.concatenate([batch.chip(c)[2][:per] for c in same], axis=0))
    el = timed(d0, S, Q, thr)
    out['first%d_of_each_%d_chips' % (per, len(same))] = round(S.shape[1] / el, 1)
    print('first-of-each', S.shape[1], round(S.shape[1] / el, 1), flush=True)

    class A:
        cpu_seconds, cpu_min_pixels = 12.0, 20000
    out['round6_cpu_baseline'] = bench.cpu_baseline(batch, A)
    print(out)


if __name__ == '__main__':
    main()
