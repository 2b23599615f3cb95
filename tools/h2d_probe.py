#!/usr/bin/env python3
"""Developer probe: PCIe copy bandwidth on the GPU box (torch pinned tensors vs the library's
pinned ChipBatch uploads), and the streaming leg's per-batch phase times.  Prints JSON."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'lcmap-firebird_amd')]

import numpy as np  # noqa: E402


def torch_bw(nbytes, reps=3):
    import torch
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d = torch.empty(nbytes, dtype=torch.uint8, device='cuda')
    out = {}
    for name, fn in (('h2d', lambda: d.copy_(h, non_blocking=True)), ('d2h', lambda: h.copy_(d, non_blocking=True))):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        out[name + '_gbs'] = nbytes * reps / (time.perf_counter() - t) / 1e9
    return out


def main():
    res = {}
    for mb in (64, 512, 2048):
        res['torch_%dMB' % mb] = torch_bw(mb << 20)
    import bench
    import ccdgpu
    from ccdgpu import synth
    cfg = synth.config(3)
    ids = list(range(8))
    page = bench.build_batch(cfg, ids)
    pin = bench.prefix_batch(page, len(ids), True)
    ctx = ccdgpu.Context(0)
    # upload only: stage into slot 0 and wait for the device
    for label, b in (('pinned', pin), ('pageable', page)):
        ctx.stage_slot_chips(0, b)
        ctx.synchronize()
        t = time.perf_counter()
        ctx.stage_slot_chips(0, b)
        ctx.synchronize()
        res['ccdgpu_upload_%s_gbs' % label] = b.nbytes / (time.perf_counter() - t) / 1e9
        ctx.run_slot(0)
    # phases of one streaming batch
    cx = np.arange(len(ids), dtype=np.int32) * 3000
    cy = np.zeros(len(ids), dtype=np.int32)
    ctx.stage_slot_chips(0, pin)
    t0 = time.perf_counter()
    ctx.run_slot(0)
    t1 = time.perf_counter()
    off, rows, mask = ctx.fetch_batch_rows(cx, cy)
    t2 = time.perf_counter()
    st = ctx.stats()
    res['batch'] = {'chips': len(ids), 'input_gb': pin.nbytes / 1e9, 'run_slot_ms': (t1 - t0) * 1e3,
                    'detect_ms': st['detect_ms'], 'fetch_rows_ms': (t2 - t1) * 1e3,
                    'rows_mb': rows.nbytes / 1e6, 'mask_mb': mask.nbytes / 1e6}
    ctx.close()
    print(json.dumps(res))


if __name__ == '__main__':
    main()
