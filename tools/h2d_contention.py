#!/usr/bin/env python3
"""Developer probe: pinned H2D upload rate of ccdgpu_stage_slot_chips alone, two contexts
uploading at once, and uploads while another context's detection runs (the tile driver's
situation).  Prints one JSON line."""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'lcmap-firebird_amd')]


def main():
    import bench
    import ccdgpu
    from ccdgpu import synth
    cfg = synth.config(3)
    ids = list(range(8))
    pin = bench.prefix_batch(bench.build_batch(cfg, ids), len(ids), True)
    big = bench.prefix_batch(bench.build_batch(cfg, list(range(16))), 16, True)
    gb = pin.nbytes / 1e9
    reps = int(os.environ.get('REPS', '4'))
    a, b = ccdgpu.Context(0), ccdgpu.Context(0)
    res = {'batch_gb': gb}

    def uploads(ctx, n, slot0=0):
        t = time.perf_counter()
        for i in range(n):
            ctx.stage_slot_chips((slot0 + i) & 1, pin)
            ctx.synchronize()
        return time.perf_counter() - t

    uploads(a, 1)
    res['alone_gbs'] = reps * gb / uploads(a, reps)
    # two contexts uploading at once
    out = {}
    th = threading.Thread(target=lambda: out.__setitem__('b', uploads(b, reps)))
    t = time.perf_counter()
    th.start()
    ta = uploads(a, reps)
    th.join()
    res['two_ctx_total_gbs'] = 2 * reps * gb / (time.perf_counter() - t)
    # uploads while the other context detects (16 chips resident, run in a thread)
    b.stage_slot_chips(0, big)
    b.synchronize()
    done = {}

    def detect():
        t0 = time.perf_counter()
        b.run_slot(0)
        done['s'] = time.perf_counter() - t0
    th = threading.Thread(target=detect)
    th.start()
    time.sleep(0.02)
    n = 0
    t = time.perf_counter()
    while th.is_alive() and n < 64:
        a.stage_slot_chips(n & 1, pin)
        a.synchronize()
        n += 1
    dt = time.perf_counter() - t
    th.join()
    res['during_detect_gbs'] = n * gb / dt if n else None
    res['during_detect_uploads'] = n
    res['detect_s'] = done.get('s')
    # the upload alone again (after)
    res['alone_after_gbs'] = reps * gb / uploads(a, reps)
    a.close()
    b.close()
    print(json.dumps(res), flush=True)
    import torch
    if not torch.cuda.is_available():
        return
    h = torch.empty(int(gb * 1e9), dtype=torch.uint8).pin_memory()
    d = torch.empty(h.numel(), dtype=torch.uint8, device='cuda')
    d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    res['torch_pinned_gbs'] = reps * h.numel() / (time.perf_counter() - t) / 1e9
    res['env_sdma'] = os.environ.get('HSA_ENABLE_SDMA')
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
