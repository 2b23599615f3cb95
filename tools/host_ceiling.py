#!/usr/bin/env python3
"""Host encode ceiling (developer tool, GPU box): K concurrent encoder threads -- the runner's
fetch threads, each encoding its own batches of distinct tile chips into its own pinned buffer
with T OpenMP threads -- for K = 1 .. 5, T = 3 (the tile's 4 x 3 within the box's 16 CPUs).
Reports the raw input rate and the host DRAM traffic it implies (raw read + encoded write, the
encoded bytes streamed; plus the DMA's read of the encoded bytes when uploaded at the same rate),
so the per-socket memory ceiling of the tile's host side can be read off where the aggregate
stops scaling with K.

usage: host_ceiling.py [chips_per_thread] [seconds_per_point]"""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'lcmap-firebird_amd'))
import numpy as np  # noqa: E402
import ccdgpu  # noqa: E402
from ccdgpu import synth  # noqa: E402


def main():
    per = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    secs = float(sys.argv[2]) if len(sys.argv) > 2 else 6.0
    K_MAX, T = 5, 3
    cfg = synth.config(3)
    from ccdc import runner
    runner.bind_to_device_node(0)
    g = synth.DeviceGenerator(0)
    pools = []
    for k in range(K_MAX):
        b = g.batch(cfg, list(range(1000 + per * k, 1000 + per * (k + 1))), pinned=False)
        pools.append([tuple(np.array(a) for a in b.chip(j)) for j in range(b.n_chips)])
    g.close()
    drop, strict = ccdgpu.unread_drop_bits(None)
    raw_per = [sum(s.nbytes + q.nbytes for _, s, q in p) for p in pools]
    out = {'chips_per_thread': per, 'omp_threads_per_encoder': T, 'cpu_quota_threads': os.environ.get('OMP_NUM_THREADS')}
    for K in range(1, K_MAX + 1):
        stop = threading.Event()
        done = [0] * K
        sent = [0] * K

        def work(k):
            e = ccdgpu.EncodedBatch([q.shape[0] for _, _, q in pools[k]], [d.shape[0] for d, _, _ in pools[k]], pinned=True)
            while not stop.is_set():
                sent[k] += e.fill(pools[k], threads=T, drop_bits=drop, strict_bits=strict)
                done[k] += 1

        th = [threading.Thread(target=work, args=(k,)) for k in range(K)]
        t = time.perf_counter()
        for x in th:
            x.start()
        time.sleep(secs)
        stop.set()
        for x in th:
            x.join()
        el = time.perf_counter() - t
        raw = sum(done[k] * raw_per[k] for k in range(K))
        enc = sum(sent)
        out['K%d' % K] = {'raw_gbs': round(raw / el / 1e9, 1), 'encoded_gbs': round(enc / el / 1e9, 1),
                          'dram_gbs_encode': round((raw + enc) / el / 1e9, 1),
                          'dram_gbs_with_dma': round((raw + 2 * enc) / el / 1e9, 1)}
        print(K, out['K%d' % K], flush=True)
    print(out)


if __name__ == '__main__':
    main()
