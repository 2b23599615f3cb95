"""The tile driver (ccdc.runner; reference core.changedetection, ccdc/core.py:78-123) on CPU:
the dynamic chip queue, the two-slot worker pipeline and the gather on rank 0, with the C oracle
standing in for the device (tests/rows_util.OracleContext).  The world-size-2 gloo run shares
one queue across two ranks through the process group's store; its gathered per-chip results must
equal a single-process run's, whatever chip went to which rank."""
import json
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TILE = os.path.join(ROOT, 'tests', 'golden', 'chipmunk', 'tile_response.json')
N_PIX = 16
N_CHIPS = 10


def tile():
    with open(TILE) as f:
        return json.load(f)


def source(pos):
    import ccdgpu
    from ccdgpu import synth
    cfg = synth.config(3)  # base-cadence and sidelap chips (two observation counts)
    return ccdgpu.ChipBatch.from_chips([synth.chip(cfg, p, 0, N_PIX) for p in pos])


def test_tile_fixture_is_the_reference_grid():
    t = tile()
    assert len(t['chips']) == 2500 and t['chips'][0] == [t['ulx'], t['uly']]


def test_local_queue_hands_out_each_position_once():
    from ccdc import runner
    q = runner.LocalQueue(10)
    got = [q.next(3) for _ in range(5)]
    assert got == [[0, 1, 2], [3, 4, 5], [6, 7, 8], [9], []]


def test_single_process_tile_run():
    from ccdc import runner
    from rows_util import OracleContext
    sink = runner.SummarySink(keep_rows=True)
    res = runner.changedetection(tile(), source, contexts=2, batch_chips=3, number=N_CHIPS, sink=sink,
                                 context_factory=lambda dev: OracleContext(dev, threads=2))
    t = tile()
    assert res['xys'] == tuple((int(x), int(y)) for x, y in t['chips'][:N_CHIPS])
    assert [c['pos'] for c in res['chips']] == list(range(N_CHIPS))
    assert {c['n_obs'] for c in res['chips']} == {1421, 2121}
    assert sum(st['chips'] for st in res['ranks']) == N_CHIPS
    # rows of one chip: pixel coordinates from the tile's chip coordinates
    off, rows, mask = sink.rows[4]
    cx, cy = (int(v) for v in t['chips'][4])
    assert rows['px'][off[:-1]].tolist() == [cx + 30 * (p % 100) for p in range(N_PIX)]
    assert (rows['py'][off[:-1]] == cy).all() and mask.shape == (N_PIX, res['chips'][4]['n_obs'])


def test_tile_run_stages_uploads_while_a_detection_runs():
    """With a context that runs detections asynchronously (run_slot_begin / run_done /
    run_slot_end, as ccdgpu.Context), the worker uploads the batches its fetch thread finishes
    while a detection runs, never into the running slot, and the rows are those of the plain
    synchronous run."""
    from ccdc import runner
    from rows_util import OracleContext, SplitOracleContext
    made = []

    def split(dev):
        made.append(SplitOracleContext(dev, threads=2, run_time=0.2))
        return made[-1]

    sink = runner.SummarySink(keep_rows=True)
    res = runner.changedetection(tile(), source, contexts=2, batch_chips=1, number=N_CHIPS, sink=sink,
                                 context_factory=split)
    ref = runner.changedetection(tile(), source, contexts=1, batch_chips=3, number=N_CHIPS,
                                 context_factory=lambda dev: OracleContext(dev, threads=2))
    assert [c['digest'] for c in res['chips']] == [c['digest'] for c in ref['chips']]
    assert sum(c.staged_during_run for c in made) > 0


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank(rank, world, port, q):
    sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'oracle'), os.path.join(ROOT, 'lcmap-firebird_amd')]
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from ccdc import runner
    from rows_util import OracleContext
    # rank 1 is slow: the shared queue must hand most chips to rank 0
    delay = 0.0 if rank == 0 else 4.0
    res = runner.changedetection(tile(), source, contexts=1, batch_chips=1, number=N_CHIPS,
                                 context_factory=lambda dev: OracleContext(dev, threads=2, delay=delay))
    q.put((rank, res))
    dist.destroy_process_group()


def test_tile_run_world2_shares_one_queue_and_gathers_on_rank0():
    import torch.multiprocessing as mp
    from ccdc import runner
    from rows_util import OracleContext
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[1] is None  # only rank 0 receives the gather
    res = out[0]
    assert [c['pos'] for c in res['chips']] == list(range(N_CHIPS))
    by_rank = {st['rank']: st['chips'] for st in res['ranks']}
    assert sum(by_rank.values()) == N_CHIPS and by_rank[0] > by_rank[1] >= 1
    # same per-chip results as one process detecting the whole tile alone
    ref = runner.changedetection(tile(), source, contexts=1, batch_chips=4, number=N_CHIPS,
                                 context_factory=lambda dev: OracleContext(dev, threads=2))
    assert [c['digest'] for c in res['chips']] == [c['digest'] for c in ref['chips']]
    assert res['xys'] == ref['xys']


def _failing_rank(rank, world, port, q):
    sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'oracle'), os.path.join(ROOT, 'lcmap-firebird_amd')]
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group('gloo', rank=rank, world_size=world, timeout=__import__('datetime').timedelta(seconds=120))
    from ccdc import runner
    from rows_util import OracleContext
    fail = RuntimeError('injected device failure') if rank == 1 else None
    try:
        runner.changedetection(tile(), source, contexts=1, batch_chips=1, number=N_CHIPS,
                               context_factory=lambda dev: OracleContext(dev, threads=2, fail=fail))
        q.put((rank, 'no error'))
    except runner.TileError as e:
        q.put((rank, ('TileError', e.rank, str(e))))
    except Exception as e:
        q.put((rank, (type(e).__name__, str(e))))
    dist.destroy_process_group()


def test_tile_run_world2_reports_a_failed_rank_without_hanging():
    """A worker failure on rank 1 reaches rank 0 as a TileError naming rank 1 and the cause;
    rank 1 raises its own error; neither rank waits for the process-group timeout."""
    import time
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    t = time.time()
    procs = [ctx.Process(target=_failing_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[0][0] == 'TileError' and out[0][1] == 1 and 'injected device failure' in out[0][2], out
    assert out[1] == ('RuntimeError', 'injected device failure'), out
    assert time.time() - t < 100


def test_runner_rejects_an_upload_depth_past_the_slots():
    from ccdc import runner
    from rows_util import OracleContext
    with pytest.raises(ValueError, match='upload_depth'):
        runner.changedetection(tile(), source, contexts=1, batch_chips=1, number=2, upload_depth=4,
                               context_factory=lambda dev: OracleContext(dev, threads=1))


def test_tail_batches_shrink_near_the_end_of_the_queue():
    from ccdc import runner
    q = runner.LocalQueue(40)
    assert runner._pull_size(q, 8, 16) == 8
    q.next(30)
    assert runner._pull_size(q, 8, 16) == 2


def test_pixel_sample_checker_passes_oracle_rows_and_flags_a_corrupted_one():
    """tests/tile_sample.py (the sampled-pixel parity behind the GPU full-size tile test and the
    bench's tile.parity_sample): rows from an oracle-backed run compare equal; a changed break day
    and a flipped mask bit are reported as integer mismatches."""
    from ccdc import runner
    from ccdgpu import synth
    from rows_util import OracleContext
    import tile_sample
    sink = tile_sample.PixelSampleSink(lambda pos: tile_sample.stratified(pos, 4, n_pix=N_PIX, width=N_PIX))
    runner.changedetection(tile(), source, contexts=2, batch_chips=2, number=6, sink=sink,
                           context_factory=lambda dev: OracleContext(dev, threads=2))

    def inputs(pos, pixels):
        d, s, q = synth.chip(synth.config(3), pos, 0, N_PIX)
        return d, s[:, pixels], q[pixels]

    out = tile_sample.check(sink, inputs, threads=4)
    assert out['pixels'] == 24 and out['chips'] == 6
    assert out['int_mismatches'] == 0 and out['float_mismatches'] == 0, out
    cx, cy, n_obs, keep = sink.samples[3]
    px = sorted(keep)[1]
    rows, mask = keep[px]
    rows['bday'][0] += 1
    mask = mask.copy()
    mask[0] ^= 1
    keep[px] = (rows, mask)
    px2 = sorted(keep)[2]
    keep[px2] = (keep[px2][0], keep[px2][1] ^ np.uint32(4))
    out = tile_sample.check(sink, inputs, threads=4)
    assert out['int_mismatches'] == 2, out


def _rank4(rank, world, port, q):
    sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'oracle'), os.path.join(ROOT, 'lcmap-firebird_amd')]
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from ccdc import runner
    from rows_util import OracleContext
    delay = 2.0 if rank == 3 else 0.0  # one slow rank
    res = runner.changedetection(tile(), source, contexts=1, batch_chips=1, number=24,
                                 context_factory=lambda dev: OracleContext(dev, threads=1, delay=delay))
    q.put((rank, res))
    dist.destroy_process_group()


def test_one_tile_split_over_world4_with_a_slow_rank():
    """The north-star mode (bench.py --tile-split; reference core.py:97-108): ONE tile's positions
    shared by four ranks through the store queue, one rank slow -- every position is detected
    exactly once, the slow rank takes fewer chips, and every rank's statistics carry its tail
    (seconds from the first empty-queue pull to its end) for rank 0."""
    import torch.multiprocessing as mp
    world = 4
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank4, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(out[r] is None for r in (1, 2, 3))
    res = out[0]
    assert [c['pos'] for c in res['chips']] == list(range(24))
    st = {s['rank']: s for s in res['ranks']}
    assert sorted(st) == [0, 1, 2, 3]
    assert sum(s['chips'] for s in st.values()) == 24
    assert st[3]['chips'] < max(st[r]['chips'] for r in (0, 1, 2))
    assert all('tail_seconds' in s and s['tail_seconds'] >= 0.0 for s in st.values())


def test_tile_run_through_the_batch_chain_equals_the_plain_run():
    """The runner's batch-chain path (run_slot_begin_rows / run_slot_end_rows, the device
    context's default): every batch goes through the chain and the rows equal a plain run's (the
    rows-buffer overflow of the chain is covered on the GPU, tests/test_gpu_tile.py)."""
    import ccdgpu
    from ccdc import runner
    from rows_util import ChainOracleContext, OracleContext
    made = []

    def chain(dev):
        made.append(ChainOracleContext(dev, threads=2, run_time=0.02))
        return made[-1]

    orig = ccdgpu.RowsBuffers.__init__

    def small(self, pinned=True, rows_per_pixel=0.25):
        orig(self, pinned=False, rows_per_pixel=rows_per_pixel)

    ccdgpu.RowsBuffers.__init__ = small
    try:
        res = runner.changedetection(tile(), source, contexts=2, batch_chips=2, number=N_CHIPS, encode=False,
                                     context_factory=chain)
    finally:
        ccdgpu.RowsBuffers.__init__ = orig
    ref = runner.changedetection(tile(), source, contexts=1, batch_chips=3, number=N_CHIPS, encode=False,
                                 context_factory=lambda dev: OracleContext(dev, threads=2))
    assert [c['digest'] for c in res['chips']] == [c['digest'] for c in ref['chips']]
    assert sum(c.chained for c in made) == sum(st['batches'] for st in res['ranks'])


def test_rows_copy_size_is_learned_and_an_overflow_still_returns_every_row():
    """RowsBuffers' copy size of the batch chain: the rate learned from a batch (1.25 x rows per
    pixel), not the whole room; a later batch with more rows per pixel than that takes the
    overflow path and still returns every row (ChainOracleContext follows ccdgpu.Context)."""
    import ccdgpu
    from rows_util import ChainOracleContext
    ctx = ChainOracleContext(0, threads=2, run_time=0.0)
    bufs = ccdgpu.RowsBuffers(pinned=False)
    from ccdgpu import synth
    cfg = synth.config(3)
    # 160 pixels a batch: more rows than the copy size's 64-row slack can hide
    batches = [ccdgpu.ChipBatch.from_chips([synth.chip(cfg, p, 0, 160)]) for p in (0, 1)]
    seen = []
    for k, b in enumerate(batches):
        ctx.stage_slot_chips(k % 2, b)
        ctx.run_slot_begin_rows(k % 2, [0], [0], bufs)
        off, rows, _ = ctx.run_slot_end_rows()
        seen.append((np.array(off), rows.copy()))
        assert bufs.copy_per_pixel is not None and bufs.copy_per_pixel <= bufs.rows_per_pixel
    ref = []
    for b in batches:
        ctx.stage_slot_chips(0, b)
        ctx.run_slot(0)
        o, r, _ = ctx.fetch_batch_rows([0], [0])
        ref.append((o, r))
    for (o1, r1), (o2, r2) in zip(seen, ref):
        assert np.array_equal(o1, o2) and r1.tobytes() == r2.tobytes()
    # force a copy size below the next batch's rows: the overflow path, the same rows
    bufs.copy_per_pixel = 0.01
    bufs.max_rate = 0.0
    before = ctx.overflowed
    ctx.stage_slot_chips(0, batches[1])
    ctx.run_slot_begin_rows(0, [0], [0], bufs)
    off, rows, _ = ctx.run_slot_end_rows()
    assert ctx.overflowed == before + 1
    assert rows.tobytes() == ref[1][1].tobytes()


@pytest.mark.parametrize('threads', [0, 2])
def test_parquet_sink_writes_the_reference_tables(tmp_path, threads):
    """ccdc.runner.ParquetSink through the tile driver (oracle-backed contexts): one segment /
    pixel / chip file per chip with the reference schemas' columns and Arrow storage types, the
    segment rows equal to the rows the run handed the sink, the pixel masks to its mask bits --
    written inline or on a pool of writer threads from copies of the reused buffers."""
    import pyarrow.parquet as pq
    from ccdc import runner, sink as sink_mod
    from ccdc import segment as seg_mod, pixel as pix_mod, chip as chip_mod
    from ccdgpu import abi
    from rows_util import OracleContext
    n = 4
    ref = runner.SummarySink(keep_rows=True)
    runner.changedetection(tile(), source, contexts=1, batch_chips=2, number=n, sink=ref,
                           context_factory=lambda dev: OracleContext(dev, threads=2))
    ps = runner.ParquetSink(str(tmp_path), threads=threads)
    res = runner.changedetection(tile(), source, contexts=2, batch_chips=2, number=n, sink=ps,
                                 context_factory=lambda dev: OracleContext(dev, threads=2))
    ps.close()
    assert [c['pos'] for c in res['chips']] == list(range(n))
    for pos, (cx, cy) in enumerate(res['xys']):
        off, rows, mask = ref.rows[pos]
        seg = pq.read_table(str(tmp_path / 'segment' / ('%d_%d.parquet' % (cx, cy))))
        pix = pq.read_table(str(tmp_path / 'pixel' / ('%d_%d.parquet' % (cx, cy))))
        chp = pq.read_table(str(tmp_path / 'chip' / ('%d_%d.parquet' % (cx, cy))))
        assert seg.schema.equals(sink_mod.arrow_schema(seg_mod.schema()))
        assert pix.schema.equals(sink_mod.arrow_schema(pix_mod.schema()))
        assert chp.schema.equals(sink_mod.arrow_schema(chip_mod.schema()))
        assert seg.equals(sink_mod.segment_table(cx, cy, rows))
        assert seg.num_rows == rows.shape[0]
        got_mask = np.array(pix.column('mask').to_pylist(), dtype=np.int8)
        assert np.array_equal(got_mask, np.asarray(mask, dtype=np.int8))
        assert chp.column('dates').to_pylist()[0] == sink_mod.iso_days(source([pos]).chip(0)[0]).tolist()


def test_parquet_sink_write_error_reaches_the_caller(tmp_path):
    """A background write that fails (here: the output directory is a file) is raised by the
    tile driver, not lost in the writer pool."""
    from ccdc import runner
    from rows_util import OracleContext
    bad = tmp_path / 'not_a_dir'
    bad.write_text('x')
    ps = runner.ParquetSink(str(bad), threads=2)
    with pytest.raises(Exception):
        runner.changedetection(tile(), source, contexts=1, batch_chips=2, number=2, sink=ps,
                               context_factory=lambda dev: OracleContext(dev, threads=2))
    ps.close()  # (the failed write was raised above; nothing left pending)


def test_parquet_sink_pool_bounds_the_chips_waiting_for_a_writer(tmp_path):
    """ParquetSink(threads, max_pending): with writers far slower than the hand-over (as Parquet
    encoding is against the device), at most max_pending chips' copies are queued or being
    written; the handing thread blocks instead of queueing every chip of the tile."""
    import threading
    import time
    from ccdc import runner
    ps = runner.ParquetSink(str(tmp_path), threads=2, max_pending=3)
    lock = threading.Lock()
    state = {'live': 0, 'peak': 0, 'done': 0}

    def slow_write(*args):
        with lock:
            state['live'] += 1
        time.sleep(0.02)
        with lock:
            state['live'] -= 1
            state['done'] += 1

    ps._write = slow_write
    queued = []
    orig_submit = ps._pool.submit

    def counting_submit(*a, **k):
        f = orig_submit(*a, **k)
        with lock:
            queued.append(f)
            state['peak'] = max(state['peak'], sum(1 for q in queued if not q.done()))
        return f

    ps._pool.submit = counting_submit
    seen = []
    ps.summary = lambda pos, *a: seen.append(pos)  # (the chip record is not under test here)
    d = np.arange(5, dtype=np.int64)
    off = np.array([0, 1], dtype=np.int64)
    rows = np.zeros(1, dtype=np.int32)
    mb = np.zeros((1, 1), dtype=np.uint64)
    for pos in range(12):
        ps(pos, 0, 0, d, off, rows, mb)
    ps.close()
    assert state['done'] == 12 and state['live'] == 0
    assert state['peak'] <= 3, state
    assert seen == list(range(12))
    with pytest.raises(ValueError):
        runner.ParquetSink(str(tmp_path), threads=1, max_pending=0)
