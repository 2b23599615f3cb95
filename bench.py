#!/usr/bin/env python3
"""bench.py -- pixels/s change-detected on MI355X (BASELINE.json metric), one JSON line.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Headline (``value``; SURVEY.md §8(d): P / wall time including H2D and the D2H of the packed
results; BASELINE.json configs[2], the CONUS ARD tile the metric names): every rank (one process
per GPU) change-detects one full 5000x5000-pixel tile -- 2500 DISTINCT chips of 100x100 pixels,
Landsat 4-8 1982-2017 cadence, the tile's own base-cadence (1421 obs) / sidelap (2121 obs) mix
-- through the product tile driver ``ccdc.runner.changedetection`` (reference
core.changedetection, ccdc/core.py:78-123): a dynamic chip queue shared by all ranks, two
contexts per GPU, pinned host batches uploaded while the previous batch is detected, rows packed
on the device and fetched back, per-chip summaries gathered on rank 0.  Chip ARD comes from the
device generator (ccdgpu.synth.TileSource): each batch is generated on the GPU and copied into
pinned host memory before the runner uploads it, so every chip is distinct and reaches the
detection path through host memory and PCIe like fetched ARD (its GPU time and device-to-host
copy are NOT excluded: the headline is pessimistic by that much).  A "step" = 1/K of the tile
(ceil(2500 / K) chips per rank); the K steps are timed as one changedetection call bracketed by
a barrier and a device synchronize; W warmup steps run first on chips of another tile.  Weak
scaling: one tile per GPU (rank r's tile = chips 2500 r .. 2500 r + 2499 of the generator).

``resident``: the detection hot path alone with inputs resident in HBM (64 tile chips per GPU,
one ragged batch per step, K steps), the kernel behind the ``roofline`` (counted FP64 flops per
launch / the launch's duration vs the MI355X FP64 vector peak, 78.6 TFLOP/s: the path is FP64
vector ALU, not a GEMM).  --config 2/4/5 selects the other synthetic configs for both legs.
cpu_baseline = the C restatement oracle (oracle/libccdoracle.so, "port") on a bounded sample of
the same chips on this host's cores (the box's 16-thread share of one GPU: the cgroup quota, so
more threads only time-slice); cpu_baseline_pyccd_restatement = the pyccd-structured numpy
restatement (oracle/ccd_ref.py), one worker process per core, on a fixed sample -- the
stand-in for the reference's per-pixel ccd.detect (ccdc/pyccd.py:168), not installable here.
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
    ap.add_argument('--cpu-min-pixels', type=int, default=20000, help='smallest CPU-baseline sample (pixels)')
    ap.add_argument('--restatement-pixels', type=int, default=1600,
                    help='pixels of the pyccd-structured restatement baseline sample')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-packer', action='store_true', help='skip the chip-packer (chipmunk decode) leg')
    ap.add_argument('--tile-chips', type=int, default=TILE_CHIPS, help='chips of the headline tile leg per rank')
    ap.add_argument('--no-resident', action='store_true',
                    help='tile leg only (knob sweeps): no resident leg, roofline null, no CPU baselines')
    ap.add_argument('--no-tile', action='store_true',
                    help='resident leg only (kernel A/B runs): value = the resident rate, not the headline metric')
    ap.add_argument('--tile-batch', type=int, default=6, help='chips per launch in the tile leg (6: 2.71-2.72M px/s vs 2.68-2.70M with 8, profiles/r04/tile_batch_ab.txt)')
    ap.add_argument('--tile-pool', type=int, default=64, help='generated chips behind the tile leg\'s chips (each position a date-shifted copy; ~18 GB of host memory per rank; 32 / 64 / 128: the same rate, profiles/r04/tile_pool_ab.txt)')
    ap.add_argument('--tile-contexts', type=int, default=4, help='contexts per GPU in the tile leg')
    ap.add_argument('--tile-copy-cus', type=int, default=8, help='CUs each tile context reserves for its upload stream (ccdgpu_init_copy_cus; 0 = none)')
    ap.add_argument('--tile-copy-threads', type=int, default=3, help='host threads per batch encode (or pool-chip copy) in the tile leg source (4 contexts x 3 within the box\'s 16-CPU quota)')
    ap.add_argument('--tile-no-numa', action='store_true', help='tile leg: leave host threads unbound (A/B)')
    ap.add_argument('--tile-no-encode', action='store_true',
                    help='tile leg: upload raw chips (pool copies into pinned batches) instead of the transport encoding (A/B)')
    ap.add_argument('--no-tile-lossless', action='store_true',
                    help='skip the second tile run with the lossless encoding (reported as tile_lossless)')
    ap.add_argument('--tile-encode', choices=('unread', 'lossless'), default='unread',
                    help='tile leg transport encoding: drop the band values of fill/cloud/shadow observations '
                         '(never read by the detection; default) or only of fill observations (lossless)')
    ap.add_argument('--tile-depth', type=int, default=2, help='batches each tile-leg context keeps uploaded ahead')
    ap.add_argument('--tile-split', action='store_true',
                    help='the north-star mode: ONE 2500-chip tile split over all ranks through the shared queue '
                         '(strong scaling; value = the tile\'s pixels / its wall time) instead of one tile per rank')
    ap.add_argument('--no-north-star', action='store_true',
                    help='N > 1: skip the extra one-tile-over-all-ranks run reported as north_star_tile')
    ap.add_argument('--tile-parity-pixels', type=int, default=16,
                    help='pixels per tile position re-detected by the C oracle after the timed tile run '
                         '(tile.parity_sample: 16 x 2500 = 4 x 10^4 pixels per tile, ~14 s of oracle time on 16 '
                         'threads; 0 = none)')
    ap.add_argument('--roofline-launches', type=int, default=3,
                    help='single-context launches of the resident batch timed for the roofline (per-launch duration)')
    ap.add_argument('--no-config-legs', action='store_true',
                    help='skip the short resident legs of the other synthetic configs (resident_c2 / _c4 / _c5)')
    ap.add_argument('--config-leg-chips', type=int, default=16, help='chips per GPU of each other-config resident leg')
    ap.add_argument('--config-leg-steps', type=int, default=3, help='timed steps of each other-config resident leg')
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
    ndev = ccdgpu.device_count()
    if local >= ndev and not args.share_device:
        raise SystemExit('LOCAL_RANK %d but only %d device(s) visible' % (local, ndev))
    device = local % ndev
    n_devices = min(world, ndev) if args.share_device else world

    if args.no_resident:
        tl = tile_leg(args, cfg, rank, world, device, dist)
        if rank == 0:
            print(json.dumps({'metric': 'tile leg only (knob sweep)', 'value': tl['value'], 'unit': 'pixels/s',
                              'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': tl['ms_per_step'],
                              'tile': tl, 'knobs': {'tile_batch': args.tile_batch, 'tile_contexts': args.tile_contexts, 'tile_copy_cus': args.tile_copy_cus,
                                                    'tile_depth': args.tile_depth,
                                                    'HSA_ENABLE_SDMA': os.environ.get('HSA_ENABLE_SDMA')}}),
                  file=json_out, flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return
    res = resident_leg(args, cfg, rank, world, device, dist)
    if args.no_tile:
        if rank == 0:
            res.pop('batch')
            out = {'metric': 'resident detection rate (kernel A/B run, not the headline metric)', 'value': res['value'],
                   'unit': 'pixels/s', 'n_gpus': n_devices, 'steps': args.steps, 'warmup': args.warmup,
                   'ms_per_step': res['ms_per_step'], 'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
                   'dtype': 'f64', 'data': 'synthetic', 'config': {'workload': res['workload'],
                                                                  'workload_key': res['workload_key']},
                   'roofline': res['roofline'], 'resident': res}
            print(json.dumps(out), file=json_out, flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return
    tl = tile_leg(args, cfg, rank, world, device, dist, split=args.tile_split)
    north = None
    if world > 1 and not args.tile_split and not args.no_north_star:
        # the north-star target: one tile over all ranks (BASELINE.json north_star; core.py:97-108)
        import copy
        a3 = copy.copy(args)
        a3.warmup = 0
        north = tile_leg(a3, cfg, rank, world, device, dist, split=True)
    tl_lossless = None
    if not args.no_tile_lossless and not args.tile_no_encode and args.tile_encode != 'lossless':
        # the same tile with the lossless encoding (device inputs bit-identical to the raw chips)
        import copy
        a2 = copy.copy(args)
        a2.tile_encode = 'lossless'
        tl_lossless = tile_leg(a2, cfg, rank, world, device, dist)
    others = {}
    if not args.no_config_legs:
        # BASELINE.json's other single-GPU configs (C2 sparse cadence, C4 masked / snow, C5
        # change-dense): a short resident leg each, with its own roofline and workload key
        import copy
        for k in sorted(CONFIG_NAMES):
            if k == args.config:
                continue
            a4 = copy.copy(args)
            a4.config, a4.chips, a4.steps, a4.warmup = k, args.config_leg_chips, args.config_leg_steps, 1
            a4.roofline_launches = 2
            r = resident_leg(a4, synth.config(k), rank, world, device, dist)
            r.pop('batch')
            others['resident_c%d' % k] = r
    if rank == 0:
        out = {
            'metric': 'pixels/sec change-detected (CONUS ARD tile) at 1/2/4/8 MI355X; FP64 VALU %',
            'value': tl['value'],
            'unit': 'pixels/s',
            'n_gpus': n_devices,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': tl['ms_per_step'],
            'higher_is_better': True,
            'scaling': 'strong' if args.tile_split else 'weak',
            'vs_baseline': None,
            'dtype': 'f64',
            'data': 'synthetic (Landsat 4-8 ARD, seeded; tile leg: every chip distinct -- date-shifted copies of GPU-generated pool chips)',
            'config': {
                'workload': '%s; %s (%d distinct 100x100-pixel chips per rank, %s), '
                            'PCIe-inclusive: chips uploaded from pinned host memory in the runner\'s transport encoding '
                            '(%s), detected, segment/pixel rows packed '
                            'on the device and fetched back, per-chip summaries gathered on rank 0 (ccdc.runner.changedetection); '
                            'a step = %d chips per rank' % (
                                CONFIG_NAMES[args.config],
                                'ONE full 5000x5000-pixel tile split over all %d GPUs' % world if args.tile_split
                                else 'one full 5000x5000-pixel tile per GPU', tl['chips_per_rank'],
                                ', '.join('%d chips of %d obs' % (v, k) for k, v in sorted(tl['n_obs_mix'].items())),
                                'raw upload' if args.tile_no_encode else
                                'band values of fill/cloud/shadow observations, which the detection never reads, not sent'
                                if args.tile_encode == 'unread' else 'lossless',
                                tl['chips_per_step']),
                'workload_key': 'tile%d_config%d_chips%d_pcie%s' % (args.tile_chips, args.config, tl['chips_per_rank'],
                                                                   '_split' if args.tile_split else ''),
                'synthetic_config': args.config,
                'chips_per_gpu': tl['chips_per_rank'],
                'pixels_per_chip': PIXELS_PER_CHIP,
                'n_obs_mix': tl['n_obs_mix'],
                'tile_chips': TILE_CHIPS,
                'ranks': world,
                'parallelism': 'chip-sharded x%d (one process per GPU, shared dynamic chip queue, no collective)' % world,
                'tile_split': bool(args.tile_split),
            },
            'roofline': res['roofline'],
            'value_resident': res['value'],
            'resident': res,
            'tile': tl,
        }
        out.update(others)
        if north is not None:
            out['north_star_tile'] = {k: north.get(k) for k in (
                'value', 'unit', 'seconds', 'chips', 'pixels', 'chips_per_rank_done', 'tail_seconds_per_rank',
                'parity_sample')}
            out['north_star_tile']['note'] = ('one 2500-chip tile split over all %d ranks through the shared queue '
                                              '(strong scaling; the target of BASELINE.json north_star)' % world)
        if tl_lossless is not None:
            out['tile_lossless'] = {k: tl_lossless[k] for k in ('value', 'unit', 'seconds', 'transport_encoding',
                                                                 'worker_seconds_rank0')}
        if not args.no_packer:
            ctx = ccdgpu.Context(device)
            out['chip_packer'] = packer_leg(ctx, res['batch'])
            ctx.close()
        if world == 1 and not args.no_cpu_baseline:
            out['cpu_baseline'] = cpu_baseline(res['batch'], args)
            out['speedup_vs_cpu_baseline'] = out['value'] / out['cpu_baseline']['value']
            b = res['batch']
            first = {}  # the batch's first chip of each date-vector length (its cadence mix)
            for c in range(b.n_chips):
                first.setdefault(int(b.chip(c)[0].shape[0]), c)
            out['cpu_baseline_pyccd_restatement'] = restatement_baseline([b.chip(c) for c in sorted(first.values())], args)
            out['speedup_vs_pyccd_restatement'] = out['value'] / out['cpu_baseline_pyccd_restatement']['value']
        res.pop('batch')
        print(json.dumps(out), file=json_out, flush=True)
    if dist is not None:
        dist.destroy_process_group()


def resident_leg(args, cfg, rank, world, device, dist, batch=None):
    """The detection hot path alone, inputs resident in HBM: the rank's ``--chips`` tile chips
    (the tile's cadence mix, spread over the tile) staged once as ONE ragged batch; K steps of
    prep + detect + scan + scatter, two contexts alternating so a launch overlaps the previous
    one's tail.  Behind the roofline."""
    import ccdgpu
    ids = chip_ids(rank, args.chips, world, lambda c: synth_nobs(cfg, c))
    if batch is None:
        batch = build_batch(cfg, ids)
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
    elapsed = max_over_ranks(elapsed, dist)
    det_avg = float(np.mean(det_ms))
    dev_avg = float(np.mean(dev_ms))
    # per-launch time behind the roofline: launches of ONE context, back to back, nothing else on
    # the device -- the HIP-event duration of each detection launch on the stream it is launched
    # on, averaged (= rocprofv3's average dispatch duration of a single-context run:
    # profiles/<round>/kernel_stats*.csv).  With two contexts a launch overlaps the other's tail
    # and its duration is inflated, so the timed steps above are not used for it.
    rl_ms, rl_dev = [], []
    for _ in range(max(1, args.roofline_launches)):
        ctx.run()
        st = ctx.stats()
        rl_ms.append(st['detect_ms'])
        rl_dev.append(st['detect_ms_device'])
        flops = st['flops']
    for c in ctxs:
        c.close()
    value = world * batch.total_pixels * args.steps / elapsed
    launch_ms = float(np.mean(rl_ms))
    achieved_tf = flops / (launch_ms * 1e-3) / 1e12
    mix = cadence_mix(batch)
    workload_key = 'config%d_chips%d_mix%s' % (args.config, len(ids), '-'.join('%dx%d' % (k, v) for k, v in sorted(mix.items())))
    pmc_file, pmc = pmc_record(workload_key)
    traffic = pmc.get('hbm_bytes_per_launch')
    pmc_c = pmc.get('counters', {})
    # occupancy of the persistent launch: its resident wave slots over the SIMDs (4 per CU), and
    # the same from the PMC pass (SQ_WAVES per launch); FP64 share of the VALU instructions
    n_cu = last.get('n_cu')
    waves_per_simd = last.get('wave_slots', 0) / (4.0 * n_cu) if n_cu else None
    f64 = sum(pmc_c.get(k, 0.0) for k in ('SQ_INSTS_VALU_ADD_F64', 'SQ_INSTS_VALU_FMA_F64', 'SQ_INSTS_VALU_MUL_F64',
                                          'SQ_INSTS_VALU_TRANS_F64'))
    fp64_share = f64 / pmc_c['SQ_INSTS_VALU'] if pmc_c.get('SQ_INSTS_VALU') else None
    pmc_waves = pmc_c['SQ_WAVES'] / (4.0 * n_cu) if pmc_c.get('SQ_WAVES') and n_cu else None
    wait_share = pmc_c.get('SQ_WAIT_ANY/SQ_WAVE_CYCLES')
    hw = hardware_fp64(pmc_c, launch_ms, n_cu)
    return {
        'value': value, 'unit': 'pixels/s', 'steps': args.steps, 'ms_per_step': elapsed / args.steps * 1e3,
        'workload': '%s; %d tile chips per GPU spread evenly over the tile (chip %d, %d, ..., %d; %s), one ragged batch '
                    'per step, inputs resident in HBM' % (
                        CONFIG_NAMES[args.config], len(ids), ids[0], ids[1] if len(ids) > 1 else ids[0], ids[-1],
                        ', '.join('%d chips of %d obs' % (v, k) for k, v in sorted(mix.items()))),
        'workload_key': workload_key, 'chips_per_gpu': len(ids), 'contexts_per_gpu': len(ctxs), 'n_obs_mix': mix,
        'mean_n_obs': float(np.mean(batch.n_obs)),
        'roofline': {
            'bound': 'fp64-valu',
            'achieved': achieved_tf,
            'peak': FP64_PEAK_TFLOPS,
            'unit': 'TFLOP/s',
            'frac': achieved_tf / FP64_PEAK_TFLOPS,
            'traffic': traffic,
            'kernel': {'w1': 'ccd_detect', 'w2': 'ccd_detect_w2', 'w3': 'ccd_detect_w3'}.get(
                os.environ.get('CCDGPU_KERNEL', 'w4'), 'ccd_detect_w4'),
            'workload_key': workload_key,
            'traffic_note': 'traffic = HBM bytes per launch from rocprofv3 --pmc (profiles/pmc_detect.json, same workload_key), else null',
            'kernel_ms_per_launch': launch_ms,
            'kernel_ms_per_launch_note': 'mean HIP-event duration of %d single-context launches (launching stream)' % len(rl_ms),
            'kernel_ms_single_context_launches': [round(x, 3) for x in rl_ms],
            'kernel_ms_single_context_device_clock': float(np.mean(rl_dev)),
            'kernel_ms_hip_events_timed_steps': det_avg,
            'kernel_ms_device_clock_timed_steps': dev_avg,
            'wall_ms_per_launch': elapsed * 1e3 / args.steps,
            'flops_per_launch': flops,
            'algorithmic_bytes_per_launch': alg_bytes,
            'algorithmic_hbm_gbs': alg_bytes / (launch_ms * 1e-3) / 1e9,
            'hbm_peak_gbs': HBM_PEAK_GBS,
            'traffic_gbs': traffic / (launch_ms * 1e-3) / 1e9 if traffic else None,
            'traffic_gbs_note': 'PMC HBM bytes per launch / kernel_ms_per_launch (L2-to-fabric traffic incl. '
                                'Infinity-Cache hits, profiles/pmc_detect.json)',
            'waves_per_simd': waves_per_simd,
            'waves_per_simd_pmc': pmc_waves,
            'waves_note': 'resident persistent waves / (4 SIMDs x CUs): launch configuration (ccdgpu_stats.wave_slots); '
                          '_pmc = SQ_WAVES per launch of the PMC pass',
            'fp64_share_of_valu': fp64_share,
            'wait_share_of_wave_cycles': wait_share,
            'pmc_record': pmc_file,
            'hw_fp64_lane_flops': hw.get('lane_flops'),
            'hw_fp64_frac': hw.get('frac'),
            'valu_busy': hw.get('valu_busy'),
            'valu_issue_model': hw.get('valu_issue_model'),
            'hw_note': hw.get('note'),
        },
        'segments_per_step': segs * world,
        'prep_ms_per_launch': float(np.mean(prep_ms)),
        'batch': batch,
    }


def pmc_record(workload_key):
    """(file name, record) of the committed PMC pass (profiles/pmc_*.json, written by
    tools/pmc_summary.py --write) taken on the same workload key, or (None, {})."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, 'profiles', 'pmc_*.json')))
    # pmc_detect.json (the C3 headline key) first, then the per-config records
    paths.sort(key=lambda p: os.path.basename(p) != 'pmc_detect.json')
    for p in paths:
        try:
            rec = json.load(open(p))
        except (OSError, ValueError):
            continue
        if isinstance(rec, dict) and rec.get('workload') == workload_key:
            return os.path.relpath(p, ROOT), rec
    return None, {}


def hardware_fp64(c, launch_ms, n_cu):
    """What the FP64 pipe really issued, from the PMC pass of the same workload key (beside the
    op-count frac, which credits modelled flops -- e.g. the closest-DOY work the comparison-rmse
    bounds skip, DESIGN.md §4 "Roofline"):
      lane_flops = 64 x (ADD + MUL + 2 FMA + TRANS)_F64 wave instructions (every lane counted, as if
                   EXEC were full: an upper bound of the lane flops the pipe did);
      frac       = lane_flops / the un-profiled launch duration / the FP64 vector peak;
      valu_busy  = SQ_ACTIVE_INST_VALU (quad-cycles, summed over waves) x 4 / (SIMDs x the launch's
                   cycles, GRBM_GUI_ACTIVE / 8 XCDs): share of SIMD cycles with a VALU issue;
      valu_issue_model = (4 cycles per FP64 + 2 per other VALU wave instruction) / SIMD cycles."""
    if not c or not launch_ms:
        return {}
    f64 = {k: c.get('SQ_INSTS_VALU_%s_F64' % k, 0.0) for k in ('ADD', 'MUL', 'FMA', 'TRANS')}
    lane = 64.0 * (f64['ADD'] + f64['MUL'] + 2.0 * f64['FMA'] + f64['TRANS'])
    out = {'lane_flops': lane, 'frac': lane / (launch_ms * 1e-3) / (FP64_PEAK_TFLOPS * 1e12),
           'note': 'hw_fp64_lane_flops = 64 x (ADD + MUL + 2 FMA + TRANS) F64 wave instructions of the PMC pass '
                   '(full-EXEC upper bound); hw_fp64_frac = that / kernel_ms_per_launch / peak; valu_busy = '
                   'SQ_ACTIVE_INST_VALU x 4 / (4 SIMDs x CUs x GRBM_GUI_ACTIVE / 8); valu_issue_model = '
                   '(4 x F64 + 2 x other VALU instructions) / the same SIMD cycles'}
    simds = 4.0 * n_cu if n_cu else None
    cyc = c.get('GRBM_GUI_ACTIVE', 0.0) / 8.0
    if simds and cyc:
        if c.get('SQ_ACTIVE_INST_VALU'):
            out['valu_busy'] = c['SQ_ACTIVE_INST_VALU'] * 4.0 / (simds * cyc)
        if c.get('SQ_INSTS_VALU'):
            nf = sum(f64.values())
            out['valu_issue_model'] = (4.0 * nf + 2.0 * (c['SQ_INSTS_VALU'] - nf)) / (simds * cyc)
    return out


def max_over_ranks(x, dist):
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _cgroup_cpu():
    """The process cgroup's CPU accounting (cgroup v2 cpu.stat: usage and throttling, usec), or
    None: whether the box's CPU quota throttled the host side of a timed run."""
    try:
        with open('/sys/fs/cgroup/cpu.stat') as f:
            return {k: int(v) for k, v in (ln.split() for ln in f if ln.strip())}
    except (OSError, ValueError):
        return None


class _ThreadCpu(object):
    """CPU seconds of this process's threads over a timed region, by thread (the host side of the
    tile: who uses the box's CPU share).  A sampler thread reads /proc/self/task/*/stat every
    ``period`` s and keeps each thread's last reading (threads that end inside the region -- the
    runner's workers -- are counted up to their last sample); Python threads are named by
    threading.enumerate(), native threads (OpenMP encoders, the HIP runtime) by their comm."""

    def __init__(self, period=0.2):
        import threading
        self.period = period
        self._stop = threading.Event()
        self._first, self._last, self._names = {}, {}, {}
        self._tick = float(os.sysconf('SC_CLK_TCK'))
        self._th = threading.Thread(target=self._run, daemon=True, name='bench-cpu-sampler')

    def _sample(self):
        import threading
        names = {t.native_id: t.name for t in threading.enumerate() if getattr(t, 'native_id', None)}
        base = '/proc/self/task'
        initial = not self._last  # the first sample: every thread alive now counts from here
        for tid in os.listdir(base):
            try:
                with open('%s/%s/stat' % (base, tid)) as f:
                    txt = f.read()
            except OSError:
                continue
            comm = txt[txt.index('(') + 1:txt.rindex(')')]
            f = txt[txt.rindex(')') + 2:].split()
            cpu = (int(f[11]) + int(f[12])) / self._tick  # utime + stime
            t = int(tid)
            self._first.setdefault(t, cpu if initial else 0.0)
            self._last[t] = cpu
            self._names[t] = names.get(t, self._names.get(t, comm))

    def _run(self):
        while not self._stop.wait(self.period):
            self._sample()

    def start(self):
        self._sample()
        self._th.start()
        return self

    def stop(self):
        self._stop.set()
        self._th.join()
        self._sample()
        by = {}
        for t, cpu in self._last.items():
            name = self._names[t]
            # group numbered threads (ccd-worker-0, Thread-3 ...) and same-comm native threads
            key = name.rstrip('0123456789').rstrip('-_ ') or name
            by[key] = by.get(key, 0.0) + cpu - self._first.get(t, 0.0)
        total = sum(by.values())
        return {'total_s': round(total, 2),
                'by_thread_s': {k: round(v, 2) for k, v in sorted(by.items(), key=lambda kv: -kv[1]) if v >= 0.05},
                'threads_seen': len(self._last),
                'note': 'utime + stime per thread of this process over the timed tile (sampled every %.1f s; '
                        'native threads by comm: OpenMP encode threads and HIP runtime threads)' % self.period}


class _Offset(object):
    """A source whose positions are shifted by ``off`` (the warmup's chips: another tile range)."""

    def __init__(self, src, off):
        self.src, self.off = src, off

    def __call__(self, positions):
        return self.src([p + self.off for p in positions])

    @property
    def has_views(self):
        return getattr(self.src, 'has_views', hasattr(self.src, 'views'))

    def views(self, positions):
        return self.src.views([p + self.off for p in positions])

    def release(self, batch):
        self.src.release(batch)


class _KeptContext(object):
    """A context created before the timed region and lent to the runner (whose close() at the
    end of a tile would otherwise free it): the timed run measures the steady-state pipeline, not
    context creation."""

    def __init__(self, ctx):
        self._ctx = ctx

    def __getattr__(self, name):
        return getattr(self._ctx, name)

    def close(self):
        pass


def tile_leg(args, cfg, rank, world, device, dist, split=False):
    """The headline: ``--tile-chips`` distinct chips per rank (default one full 2500-chip tile)
    through ccdc.runner.changedetection with chips generated on the GPU into pinned host memory
    (ccdgpu.synth.TileSource).  Positions 0 .. world * tile_chips - 1 share one dynamic queue;
    position p is generator chip p (tile p // 2500, chip p % 2500 of it; coordinates on the
    reference grid of test/data/tile_response.json shifted one tile width per tile).  W warmup
    steps run first on chips of a separate tile range (positions offset by 10^6).  ``split``: the
    north-star mode -- ONE tile of ``--tile-chips`` positions over all ranks (strong scaling).
    After the timed run, ``--tile-parity-pixels`` pixels of every position are re-detected by the
    C oracle from the position's raw inputs (tests/tile_sample.py; the checker, outside the timing)
    and reported as ``parity_sample``."""
    import ccdgpu
    from ccdc import runner
    from ccdgpu import synth
    B = args.tile_batch
    K = max(1, args.steps)
    total = int(args.tile_chips) if split else world * int(args.tile_chips)
    per_rank = -(-total // world)
    chips_per_step = -(-per_rank // K)
    warm_total = world * min(per_rank, args.warmup * chips_per_step)
    # distinct chips: a pool of generated chips, each position a different rotation of one of them
    # (configs 3 / 5, whose chips share two date vectors); configs 2 / 4 subsample dates per chip,
    # so there every chip is generated on the GPU
    mode = 'pool' if args.config in (3, 5) else 'generate'
    # host threads and the pinned batches they fill on the GPU's NUMA node (as the runner does)
    numa_node = None
    if not args.tile_no_numa:
        import ccdgpu as _cg
        numa_node = _cg.device_numa_node(device)
        runner.bind_to_device_node(device, numa_node)
    src = synth.TileSource(cfg, device=device, batch_chips=B, mode=mode, pool_chips=args.tile_pool,
                           rotate_threads=args.tile_copy_threads)
    t_prep = time.perf_counter()
    src.prepare()
    # pinned batches in flight per context: depth + 1 (fetched or staged; the runner's slot permits)
    n_inflight = args.tile_contexts * (args.tile_depth + 1) + 1
    encode = not args.tile_no_encode
    if encode:
        # the runner's transport encoding (ccdc.runner.EncodingSource): each batch is encoded from
        # the pool chips' own arrays into pinned buffers by the fetch thread and decoded on the GPU
        esrc = runner.EncodingSource(src, threads=args.tile_copy_threads, drop=args.tile_encode)
        esrc.prefill(n_inflight, B, 10000, src.max_obs)
        src_timed = src_warm = esrc
    else:
        src.prefill(n_inflight)
        src_timed = src_warm = src
    prep_s = time.perf_counter() - t_prep
    ctxs = [ccdgpu.Context(device, copy_cus=args.tile_copy_cus) for _ in range(args.tile_contexts)]
    lent = iter([])

    def factory(dev):
        return _KeptContext(next(lent))

    def xy(p):
        t, c = divmod(p % 1000000, TILE_CHIPS)
        return (-1815585 + 3000 * (c // 50) + 150000 * t, 1064805 - 3000 * (c % 50))

    sample_sink = [None]

    def run(n, src, sample=False):
        nonlocal lent
        lent = iter(ctxs)
        sink = runner.SummarySink(digest=False)
        if sample and args.tile_parity_pixels > 0:
            sys.path.insert(0, os.path.join(ROOT, 'tests'))
            import tile_sample
            k = int(args.tile_parity_pixels)
            sink = sample_sink[0] = tile_sample.PixelSampleSink(
                lambda pos: sorted({(int(pos) * 7919 + 13 + j * 1009) % PIXELS_PER_CHIP for j in range(k)}), sink)
        xys = [xy(p) for p in range(n)]
        # (encode=False: the source is already the encoding wrapper when the leg encodes)
        return runner.changedetection(xys, src, device=device, contexts=args.tile_contexts, batch_chips=B,
                                      sink=sink, upload_depth=args.tile_depth, context_factory=factory,
                                      bind_numa=not args.tile_no_numa, encode=False)

    if warm_total:
        run(warm_total, _Offset(src_warm, 1000000))
    if dist is not None:
        dist.barrier()
    ctxs[0].synchronize()
    gen0 = src.generate_seconds
    enc0 = (esrc.bytes_raw, esrc.bytes_sent, esrc.encode_seconds) if encode else (0, 0, 0.0)
    cg0 = _cgroup_cpu()
    tcpu = _ThreadCpu().start()
    t = time.perf_counter()
    res = run(total, src_timed, sample=True)
    ctxs[0].synchronize()
    if dist is not None:
        dist.barrier()
    el = max_over_ranks(time.perf_counter() - t, dist)
    thread_cpu = tcpu.stop()
    cg1 = _cgroup_cpu()  # (before the parity checker: its oracle threads are not the tile's CPU)
    parity = None
    if sample_sink[0] is not None:
        parity = tile_parity_sample(sample_sink[0], src, cfg, mode, dist)
    gen_s = src.generate_seconds - gen0
    cg = None
    if cg0 and cg1:
        cg = {k.replace('_usec', '_s'): round((cg1[k] - cg0[k]) / 1e6, 3) for k in cg0 if k in cg1 and k.endswith('usec')}
        cg.update({k: cg1[k] - cg0[k] for k in cg0 if k in cg1 and not k.endswith('usec')})
    enc_stats = None
    if encode:
        raw_b, sent_b = esrc.bytes_raw - enc0[0], esrc.bytes_sent - enc0[1]
        enc_stats = {'upload_bytes_raw_rank0': raw_b, 'upload_bytes_sent_rank0': sent_b,
                     'sent_over_raw': round(sent_b / raw_b, 4) if raw_b else None,
                     'encode_thread_seconds_rank0': round(esrc.encode_seconds - enc0[2], 3),
                     'encoder_avx512_vbmi2': bool(ccdgpu.encode_vector_path()), 'drop': args.tile_encode,
                     'drop_bits': esrc.drop_bits, 'strict_bits': esrc.strict_bits}
    for c in ctxs:
        c.close()
    src.close()
    if encode:
        esrc.close()  # the pinned encode buffers go now, not at interpreter exit
    if res is None:
        return None
    px = sum(c['n_pix'] for c in res['chips'])
    mix = {}
    for c in res['chips']:
        mix[c['n_obs']] = mix.get(c['n_obs'], 0) + 1
    ranks = {st['rank']: st for st in res['ranks']}
    return {'value': px / el, 'unit': 'pixels/s', 'seconds': el, 'ms_per_step': el / K * 1e3, 'steps': K,
            'split': bool(split), 'parity_sample': parity,
            'chips_per_step': chips_per_step, 'chips_per_rank': per_rank, 'chips': len(res['chips']), 'pixels': px,
            'distinct_chips': len(res['chips']), 'chips_per_launch': B, 'contexts_per_gpu': args.tile_contexts,
            'upload_depth': args.tile_depth, 'ranks': world, 'n_obs_mix': mix,
            'rows': sum(c['rows'] for c in res['chips']),
            'chips_per_rank_done': {r: st['chips'] for r, st in ranks.items()},
            'tail_seconds_per_rank': {r: round(st.get('tail_seconds', 0.0), 3) for r, st in ranks.items()},
            'source_mode': mode, 'source_pool_chips': args.tile_pool if mode == 'pool' else None,
            'source_copy_threads': args.tile_copy_threads if mode == 'pool' else None,
            'gpu_numa_node': numa_node, 'host_threads_bound_to_gpu_node': not args.tile_no_numa,
            'transport_encoding': enc_stats,
            'cgroup_cpu_during_tile_s': cg,
            'thread_cpu_during_tile_rank0': thread_cpu,
            'source_prepare_seconds': round(prep_s, 2),
            'generate_seconds_rank0': round(gen_s, 3),
            'pinned_pool_batches': src.allocated,
            'worker_seconds_rank0': {k: round(v, 3) for k, v in ranks[0].items() if k.endswith('_seconds')},
            'runner_trace_rank0': ranks[0].get('trace'),  # (CCDC_RUNNER_TRACE=1 only)
            'note': 'ccdc.runner tile driver over distinct chip inputs (pool mode: %d GPU-generated chips generated before '
                    'the timed run, each tile position a copy of one of its cadence with the acquisition dates moved by a '
                    'position-dependent multiple of 16 days; generate mode: every chip generated on the GPU into pinned '
                    'host memory); %s; H2D upload overlapped with detection, device row packing, D2H of rows, gather of '
                    'per-chip summaries on rank 0' % (args.tile_pool,
                    'each batch transport-encoded by the runner\'s fetch threads straight from the chip arrays into '
                    'pinned buffers (QA as palette codes; band values of fill%s observations not sent -- %s) and '
                    'decoded on the GPU' % ('/cloud/shadow' if args.tile_encode == 'unread' else '',
                                            'never read by the detection, results identical'
                                            if args.tile_encode == 'unread' else 'lossless')
                    if encode else 'chips copied into pinned batches by the runner\'s fetch threads, uploaded raw')}


def tile_parity_sample(sink, src, cfg, mode, dist):
    """Checker, after the timed tile run: the sampled pixels of every position this rank
    detected, re-detected by the C oracle from the position's raw inputs (pool mode: the
    position's moved dates and the pool chip's ARD; generate mode: the generator's pixels) and
    compared row for row (tests/tile_sample.py); summed over ranks."""
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    import tile_sample
    from ccdgpu import synth

    def inputs(pos, pixels):
        if mode == 'pool':
            d, sp, q = src.views([pos])[0]
            return d, sp[:, pixels], q[pixels]
        parts = [synth.chip(cfg, int(pos), px, 1) for px in pixels]
        return (parts[0][0], np.concatenate([p[1] for p in parts], axis=1),
                np.concatenate([p[2] for p in parts], axis=0))

    thr, _ = host_cpus()
    t = time.perf_counter()
    out = tile_sample.check(sink, inputs, threads=thr)
    out['oracle_seconds_rank0'] = round(time.perf_counter() - t, 2)
    if dist is not None:
        import torch
        v = torch.tensor([out['pixels'], out['chips'], out['int_mismatches'], out['float_mismatches']], dtype=torch.float64)
        dist.all_reduce(v)
        m = torch.tensor([out['max_rel']], dtype=torch.float64)
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        out.update(pixels=int(v[0]), chips=int(v[1]), int_mismatches=int(v[2]), float_mismatches=int(v[3]),
                   max_rel=float(m[0]))
    out['checker'] = 'C restatement oracle (oracle/libccdoracle.so), 1 thread per position, %d threads' % thr
    return out


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


def cpu_baseline(batch, args):
    """C restatement oracle (oracle/libccdoracle.so) on a bounded pixel sample of the workload's
    chips in the tile's own cadence mix -- every date vector of the batch (base cadence and
    sidelap) gets its share of the sample in proportion to its chips -- at least
    ``--cpu-min-pixels`` pixels, OpenMP over pixels, on the box's CPU share of one GPU
    (OMP_NUM_THREADS; the cgroup quota -- every affinity CPU would only time-slice on it).
    value = all sampled pixels / the summed oracle time of the groups."""
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import oracle_ctypes
    thr, info = host_cpus()
    groups = {}
    for c in range(batch.n_chips):
        groups.setdefault(int(batch.n_obs[c]), []).append(c)

    def sample(chips, n):
        """the first n pixels of `chips` (sharing one date vector), as one (spectra, qa) pair; the
        pixels of every chip are spread over it (a stride), not its first rows only"""
        S, Q, got = [], [], 0
        per = -(-n // len(chips))
        for c in chips:
            _, s, q = batch.chip(c)
            k = min(n - got, per, s.shape[1])
            sel = np.linspace(0, s.shape[1] - 1, k).astype(np.int64) if k > 0 else np.zeros(0, np.int64)
            S.append(s[:, sel])
            Q.append(q[sel])
            got += k
            if got >= n:
                break
        return np.ascontiguousarray(np.concatenate(S, axis=1)), np.ascontiguousarray(np.concatenate(Q, axis=0))

    # probe the rate on a small mixed sample, then size the sample to ~cpu_seconds (>= the minimum)
    probe_t, probe_n = 0.0, 0
    for nobs, chips in groups.items():
        k = max(thr, 16 * thr * len(chips) // batch.n_chips)
        S, Q = sample(chips, k)
        t = time.perf_counter()
        oracle_ctypes.detect_batch(batch.chip(chips[0])[0], S, Q, threads=thr)
        probe_t += time.perf_counter() - t
        probe_n += k
    rate = probe_n / probe_t
    n = int(max(args.cpu_min_pixels, rate * args.cpu_seconds))
    n = min(n, PIXELS_PER_CHIP * batch.n_chips)
    el, done, parts = 0.0, 0, []
    for nobs, chips in sorted(groups.items()):
        k = min(PIXELS_PER_CHIP * len(chips), -(-n * len(chips) // batch.n_chips))
        S, Q = sample(chips, k)
        t = time.perf_counter()
        oracle_ctypes.detect_batch(batch.chip(chips[0])[0], S, Q, threads=thr)
        dt = time.perf_counter() - t
        el += dt
        done += k
        parts.append('%d px of %d chips of %d obs (%.1f s)' % (k, len(chips), nobs, dt))
    out = {'value': done / el, 'unit': 'pixels/s', 'cores': thr, 'kind': 'port',
           'sample': '%d pixels in the workload\'s cadence mix: %s; pixels strided over each chip; C restatement '
                     'oracle, OpenMP %d threads, %.1f s in all' % (done, '; '.join(parts), thr, el)}
    out.update(info)
    return out


_RESTATEMENT_WORKER = r"""
import sys, time
import numpy as np
sys.path[:0] = sys.argv[1:3]
import ccd_ref
z = np.load(sys.argv[3])
d, S, Q = z['dates'], z['spectra'], z['qa']
lo, hi = int(sys.argv[4]), int(sys.argv[5])
ccd_ref.detect(d, *[S[b, lo] for b in range(7)], Q[lo])  # imports and first call outside the timing
print('ready', flush=True)
sys.stdin.readline()
for p in range(lo, hi):
    ccd_ref.detect(d, *[S[b, p] for b in range(7)], Q[p])
print('done', flush=True)
"""


def restatement_baseline(samples, args):
    """The restatement's rate over the workload's cadence mix: ``samples`` = one (dates, spectra,
    qa) chip per date-vector length of the batch; ``--restatement-pixels`` split evenly over them,
    each timed on its own (restatement_run) and the pixels and seconds summed."""
    thr, info = host_cpus()
    per = max(1, int(args.restatement_pixels) // max(1, len(samples)))
    tot_n, tot_s, parts = 0, 0.0, []
    for dates, S, Q in samples:
        n = min(per, S.shape[1])
        el, used = restatement_run(dates, S, Q, n, thr)
        tot_n += n
        tot_s += el
        parts.append('first %d pixels of a chip of %d obs (%.1f s)' % (n, dates.shape[0], el))
    out = {'value': tot_n / tot_s, 'unit': 'pixels/s', 'cores': used, 'kind': 'port',
           'label': 'pyccd-equivalent restatement (not pyccd itself)',
           'sample': '%d pixels in the workload\'s cadence mix: %s; oracle/ccd_ref.py, %d worker processes, %.1f s in all' % (
               tot_n, '; '.join(parts), used, tot_s)}
    out.update(info)
    return out


def restatement_run(dates, S, Q, n, thr):
    """pyccd-equivalent restatement (oracle/ccd_ref.py: pyccd's module structure, numpy + a port
    of scikit-learn 0.18's Lasso coordinate descent) on a fixed sample, one worker process per
    core of the box's share: the stand-in for reference pyccd's per-pixel ccd.detect at
    ccdc/pyccd.py:168 run "via multiprocessing" (pyccd itself is not installable here, SURVEY.md
    §8(c)).  Plain child processes (not a multiprocessing.Pool, whose resource tracker outlived
    the bench as a stray process): each loads the sample, runs one untimed pixel, reports ready;
    the timed region is from the common start signal to the last worker's end; every worker is
    reaped before this returns."""
    import subprocess
    import tempfile
    thr = max(1, min(thr, n))
    fd, path = tempfile.mkstemp(suffix='.npz')
    os.close(fd)
    procs = []
    try:
        np.savez(path, dates=dates, spectra=np.ascontiguousarray(S[:, :n]), qa=np.ascontiguousarray(Q[:n]))
        cuts = [n * k // thr for k in range(thr + 1)]
        env = dict(os.environ, OMP_NUM_THREADS='1', OPENBLAS_NUM_THREADS='1', MKL_NUM_THREADS='1')
        for k in range(thr):
            procs.append(subprocess.Popen(
                [sys.executable, '-c', _RESTATEMENT_WORKER, os.path.join(ROOT, 'oracle'),
                 os.path.join(ROOT, 'lcmap-firebird_amd'), path, str(cuts[k]), str(cuts[k + 1])],
                stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, env=env))
        for pr in procs:
            if pr.stdout.readline().strip() != 'ready':
                raise RuntimeError('restatement worker failed to start')
        t = time.perf_counter()
        for pr in procs:
            pr.stdin.write('go\n')
            pr.stdin.flush()
        for pr in procs:
            if pr.stdout.readline().strip() != 'done':
                raise RuntimeError('restatement worker failed')
        el = time.perf_counter() - t
    finally:
        for pr in procs:
            if pr.poll() is None:
                try:
                    pr.stdin.close()
                except OSError:
                    pass
            try:
                pr.wait(timeout=30)
            except subprocess.TimeoutExpired:
                pr.kill()
                pr.wait()
        os.unlink(path)
    return el, thr


def _stop_helpers():
    """At exit: every process this bench started must be gone before the JSON line's run ends.
    Lists any child still alive (to stderr, by pid and command line) and ends it."""
    try:
        import psutil
    except ImportError:
        return
    me = psutil.Process()
    kids = me.children(recursive=True)
    for k in kids:
        try:
            print('bench: ending leftover child process %d: %s' % (k.pid, ' '.join(k.cmdline())[:200]), file=sys.stderr)
            k.terminate()
        except psutil.Error:
            pass
    psutil.wait_procs(kids, timeout=5)
    for k in kids:
        try:
            if k.is_running():
                k.kill()
        except psutil.Error:
            pass
    # the record of who else runs as this user right now (not this process, its ancestors or its
    # children): a process the bench did not start but that a process count at the end would see
    try:
        mine = {me.pid} | {p.pid for p in me.parents()}
        others = []
        for p in psutil.process_iter(['pid', 'uids', 'cmdline', 'ppid']):
            if (p.info['pid'] in mine or not p.info['uids'] or p.info['uids'].real != os.getuid()
                    or not p.info['cmdline']):  # (kernel threads have no command line)
                continue
            others.append('%d (ppid %d): %s' % (p.info['pid'], p.info['ppid'], ' '.join(p.info['cmdline'] or [])[:120]))
        if others:
            print('bench: other processes of this user at exit: %s' % ' | '.join(others[:12]), file=sys.stderr)
    except psutil.Error:
        pass


if __name__ == '__main__':
    try:
        main()
    finally:
        _stop_helpers()
