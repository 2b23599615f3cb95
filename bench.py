#!/usr/bin/env python3
"""bench.py -- pixels/s change-detected on MI355X (BASELINE.json metric), one JSON line.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--chips B] [--config C]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[2], the CONUS ARD tile the metric names):
chips of a 5000x5000-pixel tile (2500 chips of 100x100 pixels, Landsat 4-8 1982-2017 cadence,
synthetic ARD from libccdsynth).  Each rank (one process per GPU) owns B chips of the tile
(chip ids rank*B .. rank*B+B-1 among the chips sharing the base cadence) staged in HBM; a
"step" is one pass of the full detection hot path over those B chips: per-chip date sort +
design rows, the per-pixel pyccd state machine, the per-pixel segment-count scan and the
segment CSR scatter, results left in HBM.  Chips are independent: no data-path collective,
weak scaling (fixed chips per GPU).  The timed region is bracketed by a barrier and a device
synchronize on both sides; the reported time is the max over ranks.

value = total pixels of all ranks / time.  roofline = counted FP64 flops of the detection
kernel per launch / its HIP-event duration vs the MI355X FP64 peak (78.6 TFLOP/s; the path is
FP64 vector ALU, not a GEMM).  cpu_baseline = the C restatement oracle (oracle/libccdoracle.so,
"port") on a bounded sample of the same chips, on this host's cores.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'lcmap-firebird_amd'))

import numpy as np  # noqa: E402

FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 vector (spec)
HBM_PEAK_GBS = 8000.0     # MI355X HBM3E (spec)
PIXELS_PER_CHIP = 10000
TILE_CHIPS = 2500


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--chips', type=int, default=64, help='chips per GPU per step')
    ap.add_argument('--config', type=int, default=3, help='synthetic config (2, 3, 4 or 5)')
    ap.add_argument('--contexts', type=int, default=2,
                    help='contexts per GPU running steps concurrently (each stages the same chips)')
    ap.add_argument('--cpu-seconds', type=float, default=12.0, help='target CPU-baseline sample time')
    ap.add_argument('--cpu-threads', type=int, default=16)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-packer', action='store_true', help='skip the chip-packer (chipmunk decode) leg')
    ap.add_argument('--no-stream', action='store_true', help='skip the end-to-end (PCIe-inclusive) streaming leg')
    ap.add_argument('--share-device', action='store_true',
                    help='rehearsal only: ranks beyond the device count share devices (LOCAL_RANK mod count)')
    return ap.parse_args()


def chip_ids(cfg, rank, chips, synth):
    """B chip ids of this rank that share the tile's base (non-sidelap) date vector, so the B
    chips stage as one batch.  Rank r takes the r-th run of B such chips of the tile."""
    base_n = synth.dates(cfg, 0).shape[0]
    found = []
    for c in range(TILE_CHIPS):
        if synth.dates(cfg, c).shape[0] == base_n:
            found.append(c)
        if len(found) >= (rank + 1) * chips:
            break
    return found[rank * chips:(rank + 1) * chips]


def main():
    args = parse()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus and 'WORLD_SIZE' in os.environ:
        print('warning: --gpus %d but WORLD_SIZE %d' % (args.gpus, world), file=sys.stderr)
    dist = None
    json_out = sys.stdout
    if world > 1:
        # gloo's native connection log goes to fd 1; keep stdout for the one JSON line
        sys.stdout.flush()
        json_out = os.fdopen(os.dup(1), 'w')
        os.dup2(2, 1)
        import torch.distributed as dist
        dist.init_process_group('gloo', rank=rank, world_size=world)

    import ccdgpu
    from ccdgpu import synth

    cfg = synth.config(args.config)
    ids = chip_ids(cfg, rank, args.chips, synth)
    dates = synth.dates(cfg, ids[0])
    n_obs = dates.shape[0]
    D = np.empty((len(ids), n_obs), np.int64)
    S = np.empty((len(ids), 7, PIXELS_PER_CHIP, n_obs), np.int16)
    Q = np.empty((len(ids), PIXELS_PER_CHIP, n_obs), np.uint16)
    for j, c in enumerate(ids):
        d, s, q = synth.chip(cfg, c, 0, PIXELS_PER_CHIP)
        assert np.array_equal(d, dates)
        D[j], S[j], Q[j] = d, s, q

    ndev = ccdgpu.device_count()
    if local >= ndev and not args.share_device:
        raise SystemExit('LOCAL_RANK %d but only %d device(s) visible' % (local, ndev))
    device = local % ndev
    ctxs = [ccdgpu.Context(device) for _ in range(max(1, args.contexts))]
    for c in ctxs:
        c.stage(D, S, Q)
    ctx = ctxs[0]

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        for c in ctxs:
            c.run()
    barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    det_ms, dev_ms, prep_ms = [], [], []
    last = {}

    def steps_on(c, k):
        # k steps on context c (ctypes releases the GIL: contexts run concurrently)
        for _ in range(k):
            c.run()
            st = c.stats()
            det_ms.append(st['detect_ms'])
            dev_ms.append(st['detect_ms_device'])
            prep_ms.append(st['prep_ms'])
            last.update(st)

    if len(ctxs) == 1:
        steps_on(ctx, args.steps)
    else:
        import threading
        share = [args.steps // len(ctxs) + (1 if i < args.steps % len(ctxs) else 0) for i in range(len(ctxs))]
        th = [threading.Thread(target=steps_on, args=(c, k)) for c, k in zip(ctxs, share)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    flops, segs, alg_bytes = last['flops'], last['segments'], last['bytes']
    ctx.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    pixels_total = world * len(ids) * PIXELS_PER_CHIP * args.steps
    value = pixels_total / elapsed
    det_avg = float(np.mean(det_ms))
    dev_avg = float(np.mean(dev_ms))
    # per-launch time behind the roofline: the HIP-event launch duration on the launching stream;
    # with concurrent contexts a launch can queue behind the other context's kernel (counted by
    # its events), so there the kernel's own execution window on the device clock is used
    launch_ms = det_avg if len(ctxs) == 1 else dev_avg
    achieved_tf = flops / (launch_ms * 1e-3) / 1e12
    traffic = None
    pmc_path = os.path.join(ROOT, 'profiles', 'pmc_detect.json')
    if os.path.exists(pmc_path):
        try:
            pmc = json.load(open(pmc_path))
            if pmc.get('workload') == 'config%d_chips%d_nobs%d' % (args.config, args.chips, n_obs):
                traffic = pmc.get('hbm_bytes_per_launch')
        except Exception:
            traffic = None

    out = {
        'metric': 'pixels/sec change-detected (CONUS ARD tile) at 1/2/4/8 MI355X; FP64 VALU %',
        'value': value,
        'unit': 'pixels/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': elapsed / args.steps * 1e3,
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'f64',
        'data': 'synthetic (libccdsynth Landsat 4-8 ARD chips, seeded)',
        'config': {
            'workload': 'C3: CONUS ARD tile chips (100x100 px, L4-L8 1982-2017 cadence, %d obs/pixel), %d chips per GPU per step' % (n_obs, len(ids)),
            'synthetic_config': args.config,
            'chips_per_gpu': len(ids), 'contexts_per_gpu': len(ctxs),
            'pixels_per_chip': PIXELS_PER_CHIP,
            'n_obs': n_obs,
            'tile_chips': TILE_CHIPS,
            'parallelism': 'chip-sharded x%d (one process per GPU, no collective)' % world,
        },
        'roofline': {
            'bound': 'mfma',
            'compute': 'fp64-valu',
            'achieved': achieved_tf,
            'peak': FP64_PEAK_TFLOPS,
            'unit': 'TFLOP/s',
            'frac': achieved_tf / FP64_PEAK_TFLOPS,
            'traffic': traffic,
            'kernel': {'w1': 'ccd_detect', 'w2': 'ccd_detect_w2'}.get(os.environ.get('CCDGPU_KERNEL', 'w3'), 'ccd_detect_w3'),
            'traffic_note': 'traffic = HBM bytes per launch from rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + WRITE_SIZE (profiles/pmc_detect.json); mostly per-wave scratch (compacted period, closest-DOY buckets) re-read from HBM',
            'kernel_ms_per_launch': launch_ms,
            'kernel_ms_hip_events': det_avg,
            'kernel_ms_device_clock': dev_avg,
            'wall_ms_per_launch': elapsed * 1e3 / args.steps,
            'flops_per_launch': flops,
            'algorithmic_bytes_per_launch': alg_bytes,
            'algorithmic_hbm_gbs': alg_bytes / (launch_ms * 1e-3) / 1e9,
            'hbm_peak_gbs': HBM_PEAK_GBS,
        },
        'segments_per_step': segs * world,
        'prep_ms_per_launch': float(np.mean(prep_ms)),
    }

    if rank == 0 and not args.no_stream:
        out['end_to_end'] = stream_leg(ctx, D[:16], S[:16], Q[:16])  # pinned copies bounded
    if rank == 0 and not args.no_packer:
        out['chip_packer'] = packer_leg(ctx, D[0], S[0], Q[0])
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out['cpu_baseline'] = cpu_baseline(S[0], Q[0], dates, args)
        out['speedup_vs_cpu_baseline'] = value / out['cpu_baseline']['value']
    if rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def stream_leg(ctx, D, S, Q, batches=6):
    """End-to-end rate from pinned host memory (never ``value``): each batch = the bench's chips,
    uploaded, detected and its CSR results fetched back.  'sequential' runs upload -> detect ->
    fetch one after another (pageable ccdgpu_stage); 'overlapped' uploads batch i+1 on the copy
    stream (ccdgpu_stage_slot, pinned buffers) while batch i is detected."""
    import ccdgpu
    n_chips = D.shape[0]
    pins = []
    for _ in range(2):
        arrs = tuple(ccdgpu.pinned_empty(x.shape, x.dtype) for x in (D, S, Q))
        for dst, src in zip(arrs, (D, S, Q)):
            dst[...] = src
        pins.append(arrs)
    px = n_chips * PIXELS_PER_CHIP * batches
    t = time.perf_counter()
    for i in range(batches):
        ctx.stage(D, S, Q)
        ctx.run()
        for c in range(n_chips):
            ctx.fetch(c)
    seq = time.perf_counter() - t
    t = time.perf_counter()
    ctx.stage_slot(0, *pins[0])
    for i in range(batches):
        if i + 1 < batches:
            ctx.stage_slot((i + 1) & 1, *pins[(i + 1) & 1])
        ctx.run_slot(i & 1)
        for c in range(n_chips):
            ctx.fetch(c)
    ovl = time.perf_counter() - t
    return {'unit': 'pixels/s', 'batches': batches, 'chips_per_batch': n_chips,
            'input_bytes_per_batch': int(D.nbytes + S.nbytes + Q.nbytes),
            'sequential_pageable': px / seq, 'overlapped_pinned': px / ovl,
            'note': 'H2D of the inputs + detection + D2H of the CSR results; not the headline value'}


def packer_leg(ctx, dates, S, Q):
    """The chip packer on one chip of the workload: its chipmunk
    payloads (base64, 8 layers x n_obs dates) decoded and pivoted on the device by
    ccd_unpack_b64.  HBM-bound byte work: bytes = text read + 16-bit values written."""
    from ccdc import chipmunk
    chips = chipmunk.chip_response(0, 0, dates, S, Q)
    d, text, offsets = chipmunk.pack_text([chipmunk.group(chips)[(0, 0)]])
    n_pix = S.shape[1]
    t = time.perf_counter()
    ctx.stage_chipmunk(d, text, offsets, n_pix)
    staged_s = time.perf_counter() - t
    ks = [ctx.stage_chipmunk(d, text, offsets, n_pix) for _ in range(3)]
    k = float(np.median(ks))
    moved = len(text) + 2 * 8 * n_pix * d.shape[1]
    return {'kernel': 'ccd_unpack_b64', 'text_bytes': len(text), 'bytes_per_launch': moved,
            'kernel_ms': k * 1e3, 'achieved_gbs': moved / k / 1e9, 'peak_gbs': HBM_PEAK_GBS,
            'frac': moved / k / 1e9 / HBM_PEAK_GBS,
            'pcie_inclusive_stage_ms': staged_s * 1e3,
            'note': 'one chip of the workload; staging = H2D of the base64 text + decode + pivot'}


def cpu_baseline(S, Q, dates, args):
    """C restatement oracle (oracle/libccdoracle.so) on a bounded pixel sample of chip 0,
    OpenMP over pixels on this host's cores."""
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import oracle_ctypes
    thr = args.cpu_threads
    n_probe = 64 * thr
    t = time.perf_counter()
    oracle_ctypes.detect_batch(dates, S[:, :n_probe], Q[:n_probe], threads=thr)
    rate = n_probe / (time.perf_counter() - t)
    n = int(min(PIXELS_PER_CHIP, max(n_probe, rate * args.cpu_seconds)))
    t = time.perf_counter()
    oracle_ctypes.detect_batch(dates, S[:, :n], Q[:n], threads=thr)
    el = time.perf_counter() - t
    return {'value': n / el, 'unit': 'pixels/s', 'cores': thr, 'kind': 'port',
            'sample': 'first %d pixels of chip 0 of the same workload (%.1f s), C restatement oracle, OpenMP' % (n, el)}


if __name__ == '__main__':
    main()
