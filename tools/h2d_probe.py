#!/usr/bin/env python3
"""Developer probe (GPU box): host-to-device copy bandwidth from pinned memory -- one stream, two
streams, four streams -- for the tile upload's sizes (the tile is upload-bound)."""
import json
import time

import torch

dev = torch.device('cuda:0')
out = {}
for size_mb in (64, 256, 1024):
    n = size_mb << 20
    srcs = [torch.empty(n, dtype=torch.uint8).pin_memory() for _ in range(4)]
    dsts = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(4)]
    for ns in (1, 2, 4):
        streams = [torch.cuda.Stream() for _ in range(ns)]
        reps = max(2, 4096 // size_mb)
        for _ in range(2):  # warm
            for i in range(ns):
                with torch.cuda.stream(streams[i]):
                    dsts[i].copy_(srcs[i], non_blocking=True)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for r in range(reps // ns):
            for i in range(ns):
                with torch.cuda.stream(streams[i]):
                    dsts[i].copy_(srcs[i], non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        gbs = (reps // ns) * ns * n / dt / 1e9
        out['%dMB_x%d_streams' % (size_mb, ns)] = round(gbs, 2)
        print(size_mb, 'MB', ns, 'streams', round(gbs, 2), 'GB/s', flush=True)
print(json.dumps(out))
