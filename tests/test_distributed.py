"""Multi-process path on CPU (gloo, world_size 2): bench.py's chip sharding gives every rank a
disjoint set of the tile's chips (in tile order, so each rank gets the tile's cadence mix), and
the barrier + max-over-ranks timing reduction behaves as the driver contract requires.  No GPU:
the detection itself is replaced by a timed no-op (the product tile runner's queue and gather
are covered by tests/test_tile.py)."""
import os
import socket
import sys

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, 'lcmap-firebird_amd')]
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import bench
    import torch
    from ccdgpu import synth
    cfg = synth.config(3)
    ids = bench.chip_ids(rank, 3, world)
    n = {synth.dates(cfg, c).shape[0] for c in ids}
    elapsed = torch.tensor([0.1 * (rank + 1)], dtype=torch.float64)
    dist.barrier()
    dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    q.put((rank, ids, sorted(n), float(elapsed.item())))
    dist.destroy_process_group()


def test_chip_sharding_and_max_timing_world2():
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    ids0, ids1 = out[0][1], out[1][1]
    assert len(ids0) == len(ids1) == 3
    assert not set(ids0) & set(ids1)
    assert ids0 == [0, 416, 833] and ids1 == [1250, 1666, 2083]
    assert out[0][3] == out[1][3] == pytest.approx(0.2)
