#!/usr/bin/env python3
"""bench.py -- pixels/s change-detected on MI355X (BASELINE.json metric), one JSON line.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--chips B] [--config C]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[2], the CONUS ARD tile the metric names):
chips of a 5000x5000-pixel tile (2500 chips of 100x100 pixels, Landsat 4-8 1982-2017 cadence,
synthetic ARD from libccdsynth).  Rank r (one process per GPU) owns B chips spread evenly over
the tile -- the tile's own mix of base-cadence (1421 obs) and sidelap (2121 obs) chips, about
half each -- staged in HBM as ONE ragged batch (ccdgpu_stage_chips).  A "step" is one
pass of the full detection hot path over those B chips: per-chip date sort + design rows, the
per-pixel pyccd state machine, the per-pixel segment-count scan and the segment CSR scatter,
results left in HBM.  Chips are independent: no data-path collective, weak scaling (fixed chips
per GPU).  The timed region is bracketed by a barrier and a device synchronize on both sides;
the reported time is the max over ranks.  --config 2/4/5 selects the other synthetic configs
(C2 1000-obs chips, C4 high-cloud/snow, C5 change-dense) over the same chip ids.

value = total pixels of all ranks / time (inputs resident in HBM).  roofline = counted FP64
flops of the detection kernel per launch / its duration vs the MI355X FP64 vector peak
(78.6 TFLOP/s; the path is FP64 vector ALU, not a GEMM).  value_e2e = the PCIe-inclusive rate of
the streaming leg (pinned uploads overlapped with detection, device-packed rows fetched back).
cpu_baseline = the C restatement oracle (oracle/libccdoracle.so, "port") on a bounded sample of
the same chips, on this host's cores; cpu_baseline_pyccd_restatement = the pyccd-structured numpy
restatement (oracle/ccd_ref.py) under multiprocessing.Pool on a fixed sample -- the stand-in
for the reference's per-pixel ccd.detect (ccdc/pyccd.py:168), which is not installable here.
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
CONFIG_NAMES = {
    2: 'C2: synthetic 100x100 chips, ~1000 obs x 7 bands + QA',
    3: 'C3: CONUS ARD tile chips (100x100 px, L4-L8 1982-2017 cadence, the tile\'s base-cadence / sidelap mix)',
    4: 'C4: high-cloud/snow stress chips (>60% masked obs)',
    5: 'C5: change-dense tile chips (breaks every ~3 yr, base-cadence / sidelap mix)',
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--chips', type=int, default=64, help='chips per GPU per step')
    ap.add_argument('--config', type=int, default=3, choices=sorted(CONFIG_NAMES), help='synthetic config')
    ap.add_argument('--contexts', type=int, default=2,
                    help='contexts per GPU running steps concurrently (each stages the same chips)')
    ap.add_argument('--cpu-seconds', type=float, default=12.0, help='target CPU-baseline sample time')
    ap.add_argument('--restatement-pixels', type=int, default=1600,
                    help='pixels of the pyccd-structured restatement baseline sample')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-packer', action='store_true', help='skip the chip-packer (chipmunk decode) leg')
    ap.add_argument('--no-stream', action='store_true', help='skip the end-to-end (PCIe-inclusive) streaming leg')
    ap.add_argument('--stream-chips', type=int, default=16, help='chips per batch of the streaming leg')
    ap.add_argument('--no-tile', action='store_true', help='skip the full-tile leg (ccdc.runner over 2500 chips)')
    ap.add_argument('--tile-chips', type=int, default=TILE_CHIPS, help='chips of the tile leg (all ranks together)')
    ap.add_argument('--tile-batch', type=int, default=8, help='chips per launch in the tile leg')
    ap.add_argument('--tile-contexts', type=int, default=2, help='contexts per GPU in the tile leg')
    ap.add_argument('--tile-depth', type=int, default=2, help='batches each tile-leg context keeps uploaded ahead')
    ap.add_argument('--share-device', action='store_true',
                    help='rehearsal only: ranks beyond the device count share devices (LOCAL_RANK mod count)')
    return ap.parse_args()


def chip_ids(rank, chips, world=1, n_obs_of=None):
    """The rank's B chips of the tile (weak scaling: B chips per rank).  Tile chips are grouped
    by observation count (base cadence / sidelap, n_obs_of(chip)); every rank takes each group's
    share of B in proportion to the group's share of the tile, evenly spaced through the group,
    so all ranks carry the tile's own cadence mix (a contiguous run of chips would not: the first
    64 chips are 2/3 sidelap)."""
    total = world * chips
    if total > TILE_CHIPS:
        raise SystemExit('%d ranks x %d chips exceeds the %d-chip tile' % (world, chips, TILE_CHIPS))
    if n_obs_of is None:
        return [(rank * chips + j) * TILE_CHIPS // total for j in range(chips)]
    groups = {}
    for c in range(TILE_CHIPS):
        groups.setdefault(n_obs_of(c), []).append(c)
    keys = sorted(groups)
    share = [chips * len(groups[k]) // TILE_CHIPS for k in keys]
    for i in sorted(range(len(keys)), key=lambda i: -len(groups[keys[i]]))[:chips - sum(share)]:
        share[i] += 1
    ids = []
    for k, s in zip(keys, share):
        g = groups[k]
        ids += [g[(rank * s + j) * len(g) // (world * s)] for j in range(s)]
    return sorted(ids)


def build_batch(cfg, ids, pinned=False):
    """The chips as one ragged ChipBatch, generated in place (libccdsynth).  With
    CCD_BENCH_CACHE=<dir> (profiling runs that start the bench several times) the generated
    buffers are kept there and reloaded instead of regenerated."""
    import ccdgpu
    from ccdgpu import synth
    nobs = [synth.dates(cfg, c).shape[0] for c in ids]
    b = ccdgpu.ChipBatch([PIXELS_PER_CHIP] * len(ids), nobs, pinned=pinned)
    cache = os.environ.get('CCD_BENCH_CACHE')
    key = None
    if cache:
        import hashlib
        key = os.path.join(cache, 'batch_%s' % hashlib.sha1(
            repr((bytes(cfg), list(ids), PIXELS_PER_CHIP)).encode()).hexdigest()[:16])
        if os.path.exists(key + '.done'):
            for name in ('dates', 'spectra', 'qa'):
                getattr(b, name)[...] = np.load('%s_%s.npy' % (key, name), mmap_mode='r')
            return b
    for j, c in enumerate(ids):
        synth.chip(cfg, c, 0, PIXELS_PER_CHIP, out=b.chip(j))
    if key:
        os.makedirs(cache, exist_ok=True)
        for name in ('dates', 'spectra', 'qa'):
            np.save('%s_%s.npy' % (key, name), np.asarray(getattr(b, name)))
        open(key + '.done', 'w').close()
    return b


def cadence_mix(batch):
    vals, counts = np.unique(batch.n_obs, return_counts=True)
    return {int(v): int(k) for v, k in zip(vals, counts)}


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
    ids = chip_ids(rank, args.chips, world, lambda c: synth.dates(cfg, c).shape[0])
    batch = build_batch(cfg, ids)

    ndev = ccdgpu.device_count()
    if local >= ndev and not args.share_device:
        raise SystemExit('LOCAL_RANK %d but only %d device(s) visible' % (local, ndev))
    device = local % ndev
    n_devices = min(world, ndev) if args.share_device else world
    ctxs = [ccdgpu.Context(device) for _ in range(max(1, args.contexts))]
    for c in ctxs:
        c.stage_chips(batch)
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

    pixels_total = world * batch.total_pixels * args.steps
    value = pixels_total / elapsed
    det_avg = float(np.mean(det_ms))
    dev_avg = float(np.mean(dev_ms))
    # per-launch time behind the roofline: the HIP-event launch duration on the launching stream;
    # with concurrent contexts a launch can queue behind the other context's kernel (counted by
    # its events), so there the kernel's own execution window on the device clock is used
    launch_ms = det_avg if len(ctxs) == 1 else dev_avg
    achieved_tf = flops / (launch_ms * 1e-3) / 1e12
    mix = cadence_mix(batch)
    workload_key = 'config%d_chips%d_mix%s' % (args.config, len(ids), '-'.join('%dx%d' % (k, v) for k, v in sorted(mix.items())))
    traffic = None
    pmc_path = os.path.join(ROOT, 'profiles', 'pmc_detect.json')
    if os.path.exists(pmc_path):
        try:
            pmc = json.load(open(pmc_path))
            if pmc.get('workload') == workload_key:
                traffic = pmc.get('hbm_bytes_per_launch')
        except Exception:
            traffic = None

    out = {
        'metric': 'pixels/sec change-detected (CONUS ARD tile) at 1/2/4/8 MI355X; FP64 VALU %',
        'value': value,
        'unit': 'pixels/s',
        'n_gpus': n_devices,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': elapsed / args.steps * 1e3,
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'f64',
        'data': 'synthetic (libccdsynth Landsat 4-8 ARD chips, seeded)',
        'config': {
            'workload': '%s; %d tile chips per GPU spread evenly over the tile (chip %d, %d, ..., %d; %s), one ragged batch per step, inputs resident in HBM' % (
                CONFIG_NAMES[args.config], len(ids), ids[0], ids[1] if len(ids) > 1 else ids[0], ids[-1],
                ', '.join('%d chips of %d obs' % (v, k) for k, v in sorted(mix.items()))),
            'workload_key': workload_key,
            'synthetic_config': args.config,
            'chips_per_gpu': len(ids), 'contexts_per_gpu': len(ctxs),
            'pixels_per_chip': PIXELS_PER_CHIP,
            'n_obs_mix': mix,
            'mean_n_obs': float(np.mean(batch.n_obs)),
            'tile_chips': TILE_CHIPS,
            'ranks': world,
            'parallelism': 'chip-sharded x%d (one process per GPU, no collective)' % world,
        },
        'roofline': {
            'bound': 'fp64-valu',
            'achieved': achieved_tf,
            'peak': FP64_PEAK_TFLOPS,
            'unit': 'TFLOP/s',
            'frac': achieved_tf / FP64_PEAK_TFLOPS,
            'traffic': traffic,
            'kernel': {'w1': 'ccd_detect', 'w2': 'ccd_detect_w2', 'w4': 'ccd_detect_w4'}.get(
                os.environ.get('CCDGPU_KERNEL', 'w3'), 'ccd_detect_w3'),
            'traffic_note': 'traffic = HBM bytes per launch from rocprofv3 --pmc (profiles/pmc_detect.json, same workload_key), else null',
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

    if not args.no_tile:
        # every rank takes part (shared dynamic queue); rank 0 gets the gathered result
        tl = tile_leg(args, cfg, rank, world, device, dist)
        if rank == 0:
            out['tile'] = tl
            out['value_e2e'] = tl['value']
    if rank == 0 and not args.no_stream:
        out['end_to_end'] = stream_leg(ctx, batch, min(args.stream_chips, batch.n_chips))
        out.setdefault('value_e2e', out['end_to_end']['overlapped_pinned'])
    if rank == 0 and not args.no_packer:
        out['chip_packer'] = packer_leg(ctx, batch)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        d, s, q = batch.chip(0)
        out['cpu_baseline'] = cpu_baseline(d, s, q, args)
        out['speedup_vs_cpu_baseline'] = value / out['cpu_baseline']['value']
        out['cpu_baseline_pyccd_restatement'] = restatement_baseline(d, s, q, args)
        out['speedup_vs_pyccd_restatement'] = value / out['cpu_baseline_pyccd_restatement']['value']
    if rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    for c in ctxs:
        c.close()
    if dist is not None:
        dist.destroy_process_group()


def tile_leg(args, cfg, rank, world, device, dist):
    """The product tile driver (ccdc.runner.changedetection; reference core.changedetection,
    ccdc/core.py:78-123) over the tile's chip grid on every rank's GPU: one dynamic chip queue
    shared by all ranks (the process group's store), two contexts per GPU each keeping two pinned
    batch uploads queued ahead of its detection, device row packing, rows fetched back per batch, per-chip
    summaries gathered on rank 0.  PCIe-inclusive.  Chip ARD comes from a pool of two
    pre-generated pinned batches of the tile's cadence mix, cycled over the tile positions, so
    host-side synthetic generation (the chipmunk fetch stand-in) stays out of the timing."""
    from ccdc import runner
    B = args.tile_batch
    ids = chip_ids(0, 2 * B, 1, lambda c: synth_nobs(cfg, c))
    pool = [build_batch(cfg, ids[k::2], pinned=True) for k in range(2)]
    tails = {}

    def source(pos):
        b = pool[(pos[0] // B) % 2]
        if len(pos) == b.n_chips:
            return b
        if len(pos) not in tails:
            tails[len(pos)] = prefix_batch(b, len(pos), True)
        return tails[len(pos)]

    xys = [(-1815585 + 3000 * (c // 50), 1064805 - 3000 * (c % 50)) for c in range(TILE_CHIPS)]
    sink = runner.SummarySink(digest=False)
    if dist is not None:
        dist.barrier()
    t = time.perf_counter()
    res = runner.changedetection(xys, source, device=device, contexts=args.tile_contexts, batch_chips=B,
                                 number=args.tile_chips, sink=sink, upload_depth=args.tile_depth)
    el = time.perf_counter() - t
    if res is None:
        return None
    px = sum(c['n_pix'] for c in res['chips'])
    mix = {}
    for c in res['chips']:
        mix[c['n_obs']] = mix.get(c['n_obs'], 0) + 1
    return {'value': px / el, 'unit': 'pixels/s', 'seconds': el, 'chips': len(res['chips']), 'pixels': px,
            'chips_per_launch': B, 'contexts_per_gpu': args.tile_contexts, 'upload_depth': args.tile_depth,
            'ranks': world, 'n_obs_mix': mix,
            'rows': sum(c['rows'] for c in res['chips']),
            'chips_per_rank': {st['rank']: st['chips'] for st in res['ranks']},
            'worker_seconds_rank0': {k: round(v, 3) for k, v in res['ranks'][0].items() if k.endswith('_seconds')},
            'note': 'ccdc.runner tile driver: shared dynamic chip queue, H2D of pinned ARD + detection + device row packing + D2H of rows + gather of per-chip summaries on rank 0; chip ARD cycled over 2 pre-generated pinned batches of the tile mix'}


def synth_nobs(cfg, c):
    from ccdgpu import synth
    return synth.dates(cfg, c).shape[0]


def prefix_batch(batch, n, pinned):
    """The first n chips of a ChipBatch (a prefix of its flat buffers) as a new batch."""
    import ccdgpu
    b = ccdgpu.ChipBatch(batch.n_pix[:n], batch.n_obs[:n], pinned=pinned)
    b.dates[...] = batch.dates[:b.dates.shape[0]]
    b.spectra[...] = batch.spectra[:b.spectra.shape[0]]
    b.qa[...] = batch.qa[:b.qa.shape[0]]
    return b


def stream_leg(ctx, batch, n, batches=6):
    """End-to-end rate (never ``value``): each batch = the first n chips of the workload (the
    tile's cadence mix) uploaded, detected and their rows packed on the device and fetched back (the product
    output: float32 segment rows + per-date pixel masks).  'sequential' runs upload -> detect ->
    fetch one after another from pageable memory; 'overlapped' uploads batch i+1 from pinned
    memory on the copy stream (ccdgpu_stage_slot_chips) while batch i is detected."""
    pins = [prefix_batch(batch, n, True) for _ in range(2)]
    page = prefix_batch(batch, n, False)
    cx = np.arange(n, dtype=np.int32) * 3000
    cy = np.zeros(n, dtype=np.int32)
    px = page.total_pixels * batches
    t = time.perf_counter()
    for i in range(batches):
        ctx.stage_chips(page)
        ctx.run()
        ctx.fetch_batch_rows(cx, cy)
    seq = time.perf_counter() - t
    t = time.perf_counter()
    ctx.stage_slot_chips(0, pins[0])
    for i in range(batches):
        if i + 1 < batches:
            ctx.stage_slot_chips((i + 1) & 1, pins[(i + 1) & 1])
        ctx.run_slot(i & 1)
        ctx.fetch_batch_rows(cx, cy)
    ovl = time.perf_counter() - t
    return {'unit': 'pixels/s', 'batches': batches, 'chips_per_batch': n,
            'input_bytes_per_batch': int(page.nbytes), 'n_obs_mix': cadence_mix(page),
            'sequential_pageable': px / seq, 'overlapped_pinned': px / ovl,
            'h2d_gbs_overlapped': page.nbytes * batches / ovl / 1e9,
            'note': 'H2D of the inputs + detection + device row packing + D2H of the rows; not the headline value'}


def packer_leg(ctx, batch):
    """The chip packer on one chip of the workload: its chipmunk
    payloads (base64, 8 layers x n_obs dates) decoded and pivoted on the device by
    ccd_unpack_b64.  HBM-bound byte work: bytes = text read + 16-bit values written."""
    from ccdc import chipmunk
    dates, S, Q = batch.chip(0)
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


def host_cpus():
    """(threads to use, description): the CPUs this process may run on, capped by the
    OMP_NUM_THREADS share the GPU box grants one GPU, plus the CPU model."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    share = int(os.environ.get('OMP_NUM_THREADS', '0') or 0)
    use = min(avail, share) if share > 0 else avail
    model = ''
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                model = line.split(':', 1)[1].strip()
                break
    except OSError:
        pass
    return use, {'cpu_model': model, 'os_cpu_count': os.cpu_count(), 'affinity_cpus': avail,
                 'omp_num_threads_share': share or None}


def cpu_baseline(dates, S, Q, args):
    """C restatement oracle (oracle/libccdoracle.so) on a bounded pixel sample of chip 0,
    OpenMP over pixels on this host's cores."""
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import oracle_ctypes
    thr, info = host_cpus()
    n_probe = 32 * thr
    t = time.perf_counter()
    oracle_ctypes.detect_batch(dates, S[:, :n_probe], Q[:n_probe], threads=thr)
    rate = n_probe / (time.perf_counter() - t)
    n = int(min(PIXELS_PER_CHIP, max(n_probe, rate * args.cpu_seconds)))
    t = time.perf_counter()
    oracle_ctypes.detect_batch(dates, S[:, :n], Q[:n], threads=thr)
    el = time.perf_counter() - t
    out = {'value': n / el, 'unit': 'pixels/s', 'cores': thr, 'kind': 'port',
           'sample': 'first %d pixels of chip 0 of the same workload (%d obs, %.1f s), C restatement oracle, OpenMP %d threads' % (
               n, dates.shape[0], el, thr)}
    out.update(info)
    return out


def _restatement_pixel(args):
    import ccd_ref
    d, s, q = args
    return len(ccd_ref.detect(d, *[s[b] for b in range(7)], q)['change_models'])


def restatement_baseline(dates, S, Q, args):
    """pyccd-equivalent restatement (oracle/ccd_ref.py: pyccd's module structure, numpy + a port
    of scikit-learn 0.18's Lasso coordinate descent) under multiprocessing.Pool on a fixed
    sample: the stand-in for reference pyccd's per-pixel ccd.detect at ccdc/pyccd.py:168 (pyccd
    itself is not installable here)."""
    import multiprocessing
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    thr, info = host_cpus()
    n = min(args.restatement_pixels, S.shape[1])
    jobs = [(dates, S[:, p].copy(), Q[p].copy()) for p in range(n)]
    ctx = multiprocessing.get_context('spawn')
    with ctx.Pool(thr) as pool:
        pool.map(_restatement_pixel, jobs[:thr])  # worker start-up and imports outside the timing
        t = time.perf_counter()
        pool.map(_restatement_pixel, jobs, chunksize=1)
        el = time.perf_counter() - t
    out = {'value': n / el, 'unit': 'pixels/s', 'cores': thr, 'kind': 'port',
           'label': 'pyccd-equivalent restatement (not pyccd itself)',
           'sample': 'first %d pixels of chip 0 of the same workload (%d obs, %.1f s), oracle/ccd_ref.py, multiprocessing.Pool(%d)' % (
               n, dates.shape[0], el, thr)}
    out.update(info)
    return out


if __name__ == '__main__':
    main()
