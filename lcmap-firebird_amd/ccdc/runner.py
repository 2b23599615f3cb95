"""ccdc.runner -- the tile driver: change detection of a whole tile's chips on the GPUs of one node.

Reference: ``core.changedetection`` (ccdc/core.py:78-123) takes a tile's chip coordinates from
``grid.tile`` (core.py:97; fixture test/data/tile_response.json: 2500 chips), splits them with
``partition_all(chunk_size)`` (core.py:98-99) and runs ``core.detect`` (core.py:53-75) per chunk:
``ids.rdd`` -> ``timeseries.rdd`` (merlin fetch, per-pixel pivot, ``repartition``,
timeseries.py:92-126) -> ``pyccd.rdd`` (one ``ccd.detect`` per pixel, pyccd.py:171-183) -> the
chip / pixel / segment writes.  Spark balances the per-pixel work dynamically (repartition and
task scheduling) and the driver collects the processed chip coordinates.

Here one process runs per GPU (a torch.distributed rank, or a plain process) and inside it
``contexts`` worker threads, each with its own ``ccdgpu.Context``.  A worker repeatedly takes
the next ``batch_chips`` chips from a ``ChipQueue`` shared by every worker of every rank -- a
dynamic queue, so chips of very different cost (sidelap vs base cadence, change-dense chips)
balance themselves across GPUs -- asks the ``source`` for their ARD as a ``ccdgpu.ChipBatch``
(the merlin/chipmunk fetch stand-in; pinned batches upload asynchronously), uploads it on the
copy stream while its previous batch is being detected, runs the detection, packs the segment /
pixel table rows on the device and fetches them in one copy (ccdgpu_fetch_batch_rows), and hands
every chip's rows to the ``sink``.  No collective touches the data path: the only cross-rank
traffic is the queue counter (the process group's key-value store) and the final gather of the
per-chip summaries on rank 0 (``gather``).
"""
import threading
import time

import numpy as np

from ccdc import logger


# --------------------------------------------------------------------------- chip queues
class LocalQueue(object):
    """Dynamic queue of tile positions 0 .. total-1 for the worker threads of one process."""

    def __init__(self, total):
        self.total = int(total)
        self._next = 0
        self._lock = threading.Lock()

    def next(self, n):
        with self._lock:
            a = self._next
            self._next = min(self.total, a + int(n))
            return list(range(a, self._next))


class StoreQueue(object):
    """Dynamic queue of tile positions shared by every rank of a torch.distributed job: one atomic
    counter in the process group's key-value store (``store.add``); every rank pulls the next
    ``n`` positions when it has capacity, so ranks that got cheap chips simply take more.  All
    ranks must construct it with the same ``name`` (``changedetection`` derives it from a call
    counter and synchronises with a barrier)."""

    def __init__(self, total, name, store=None):
        import torch.distributed as dist
        if store is None:
            from torch.distributed import distributed_c10d
            store = distributed_c10d._get_default_store()
        self.total = int(total)
        self.key = 'ccdc.runner.queue.%s' % name
        self.store = store
        self._dist = dist

    def next(self, n):
        if n <= 0:
            return []
        end = int(self.store.add(self.key, int(n)))
        a = end - int(n)
        return list(range(min(a, self.total), min(end, self.total)))


# --------------------------------------------------------------------------- sinks
def chip_checksum(row_offsets, rows, mask_bits):
    """Order-sensitive digest of one chip's rows and processing-mask bit words (for gathers and
    parity checks)."""
    import hashlib
    h = hashlib.sha1()
    h.update(np.ascontiguousarray(row_offsets, dtype=np.int64).tobytes())
    h.update(np.ascontiguousarray(rows).tobytes())
    h.update(np.ascontiguousarray(mask_bits, dtype='<u4').tobytes())
    return h.hexdigest()


class SummarySink(object):
    """Keeps one small summary per chip (position, coordinates, pixels, rows, change models,
    digest) and, with keep_rows, the rows themselves (tests / small runs)."""

    def __init__(self, keep_rows=False, digest=True):
        self.keep_rows = keep_rows
        self.digest = digest
        self.chips = []
        self.rows = {}
        self._lock = threading.Lock()

    def __call__(self, pos, cx, cy, dates, row_offsets, rows, mask_bits):
        s = {'pos': int(pos), 'cx': int(cx), 'cy': int(cy), 'n_pix': int(len(row_offsets) - 1),
             'n_obs': int(dates.shape[0]), 'rows': int(rows.shape[0]),
             'models': int(np.count_nonzero(rows['has_model'])),
             'digest': chip_checksum(row_offsets, rows, mask_bits) if self.digest else None}
        with self._lock:
            self.chips.append(s)
            if self.keep_rows:
                from ccdgpu import abi
                self.rows[int(pos)] = (np.array(row_offsets), rows.copy(),
                                       abi.unpack_mask_bits(mask_bits, dates.shape[0]))


class ParquetSink(object):
    """The offline writer: each chip's segment / pixel / chip tables (reference schemas,
    ccdc.sink) as <directory>/<table>/<cx>_<cy>.parquet, plus a SummarySink record."""

    def __init__(self, directory):
        self.directory = directory
        self.summary = SummarySink()

    def __call__(self, pos, cx, cy, dates, row_offsets, rows, mask_bits):
        from ccdc import sink
        from ccdgpu import abi
        mask = abi.unpack_mask_bits(mask_bits, dates.shape[0])
        sink.write_parquet(self.directory, sink.tables(cx, cy, dates, row_offsets, rows, mask), cx, cy)
        self.summary(pos, cx, cy, dates, row_offsets, rows, mask_bits)

    @property
    def chips(self):
        return self.summary.chips


# --------------------------------------------------------------------------- the GPU worker
def _worker(ctx, queue, source, xys, batch_chips, params, width, sink, stats, errors, depth=2):
    """One context: up to ``depth`` batches uploaded (or uploading) ahead of the one being
    detected, one upload slot each, so the PCIe link stays busy while a batch is detected and
    its rows are fetched (with one batch ahead the link idles whenever both of a GPU's contexts
    are past their upload)."""
    try:
        clock = time.perf_counter
        free = list(range(depth + 1))
        staged = []  # (slot, positions, batch), in upload order
        exhausted = False
        while True:
            while free and not exhausted:
                t0 = clock()
                pos = queue.next(batch_chips)
                if not pos:
                    exhausted = True
                    break
                batch = source(pos)
                if batch.n_chips != len(pos):
                    raise ValueError('source returned %d chips for %d positions' % (batch.n_chips, len(pos)))
                t1 = clock()
                slot = free.pop(0)
                ctx.stage_slot_chips(slot, batch, params)
                staged.append((slot, pos, batch))
                t2 = clock()
                with stats['lock']:
                    stats['source_seconds'] += t1 - t0
                    stats['stage_seconds'] += t2 - t1
            if not staged:
                break
            s, ppos, pbatch = staged.pop(0)
            t2 = clock()
            ctx.run_slot(s)
            if getattr(ctx, 'qa_error', False):
                import ccdgpu
                raise ccdgpu.QAValueError('unsupported bit-packed QA value in chips at tile positions %s' % (ppos,))
            t3 = clock()
            cx = np.array([xys[p][0] for p in ppos], dtype=np.int32)
            cy = np.array([xys[p][1] for p in ppos], dtype=np.int32)
            off, rows, mask = ctx.fetch_batch_rows(cx, cy, width)
            free.append(s)  # its rows are fetched: the slot takes the next upload
            t4 = clock()
            for c, p in enumerate(ppos):
                p0, p1 = int(pbatch.pix_off[c]), int(pbatch.pix_off[c + 1])
                r0, r1 = int(off[p0]), int(off[p1])
                d, _, _ = pbatch.chip(c)
                sink(p, int(cx[c]), int(cy[c]), d, off[p0:p1 + 1] - r0, rows[r0:r1], pbatch.mask_bits_of(mask, c))
            t5 = clock()
            with stats['lock']:
                stats['batches'] += 1
                stats['chips'] += len(ppos)
                stats['pixels'] += pbatch.total_pixels
                stats['rows'] += int(rows.shape[0])
                stats['device_seconds'] += t3 - t2
                stats['fetch_seconds'] += t4 - t3
                stats['sink_seconds'] += t5 - t4
    except BaseException as e:  # reported by detect_tile after the other workers drain
        errors.append(e)


def detect_tile(xys, source, queue, device=0, contexts=2, batch_chips=16, params=None, width=100,
                sink=None, context_factory=None, upload_depth=2):
    """Change detection of the tile chips at ``xys`` (list of (cx, cy), tile order) on one GPU.

    ``source(positions) -> ccdgpu.ChipBatch`` supplies the ARD of the chips at those tile
    positions (pinned batches upload asynchronously); ``queue`` hands out positions (LocalQueue
    for one process, StoreQueue across ranks); ``sink(pos, cx, cy, dates, row_offsets, rows,
    mask_bits)`` receives each chip's device-packed rows and its processing masks as bit words
    [n_pix][words] (ccdgpu.abi.unpack_mask_bits; default sink: a SummarySink).  Returns the sink
    and this process's statistics.  ``upload_depth``: batches each context keeps uploaded or
    uploading ahead of the one it detects (1 .. ccdgpu.UPLOAD_SLOTS - 1)."""
    if context_factory is None:
        import ccdgpu
        context_factory = ccdgpu.Context
    sink = sink if sink is not None else SummarySink()
    # per-phase host seconds summed over the workers: source (ARD fetch), stage (upload call),
    # device (run_slot: waits for the upload, detects), fetch (row packing + D2H), sink
    stats = {'lock': threading.Lock(), 'batches': 0, 'chips': 0, 'pixels': 0, 'rows': 0, 'device_seconds': 0.0,
             'source_seconds': 0.0, 'stage_seconds': 0.0, 'fetch_seconds': 0.0, 'sink_seconds': 0.0}
    errors = []
    ctxs = [context_factory(device) for _ in range(max(1, int(contexts)))]
    t0 = time.perf_counter()
    try:
        th = [threading.Thread(target=_worker, args=(c, queue, source, xys, batch_chips, params, width, sink, stats, errors,
                                                       max(1, int(upload_depth))))
              for c in ctxs]
        for t in th:
            t.start()
        for t in th:
            t.join()
    finally:
        for c in ctxs:
            c.close()
    if errors:
        raise errors[0]
    stats.pop('lock')
    stats['seconds'] = time.perf_counter() - t0
    return sink, stats


_calls = [0]


def gather(obj, dist=None):
    """All ranks' ``obj`` as a list on rank 0 (None elsewhere); [obj] without a process group.
    Uses a gloo group, so it works whatever backend the default group has."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return [obj]
    group = dist.new_group(backend='gloo')
    out = [None] * dist.get_world_size() if dist.get_rank() == 0 else None
    dist.gather_object(obj, out, dst=0, group=group)
    return out


def changedetection(tile, source, device=None, contexts=2, batch_chips=16, number=None, params=None,
                    sink=None, width=100, context_factory=None, ctx=None, upload_depth=2):
    """Change detection for a tile on every GPU of the job (reference core.changedetection,
    ccdc/core.py:78-123).

    ``tile``: {'chips': [[cx, cy], ...]} (grid.tile's response, test/data/tile_response.json) or
    a plain list of (cx, cy); ``number`` limits the chips (the reference's testing knob);
    ``source(positions) -> ChipBatch``.  Under torch.distributed every rank calls this with the
    same arguments: ranks share one dynamic chip queue and rank 0 gets the gathered result.
    Returns (on rank 0, else None) {'xys': processed chip coordinates in tile order, 'chips':
    per-chip summaries, 'ranks': per-rank statistics}."""
    try:
        import torch.distributed as dist
        dist_on = dist.is_available() and dist.is_initialized()
    except ImportError:
        dist, dist_on = None, False
    chips = tile.get('chips') if isinstance(tile, dict) else tile
    xys = [(int(c[0]), int(c[1])) for c in chips]
    if number is not None:
        xys = xys[:int(number)]
    log = logger(ctx, name=__name__)
    if dist_on and dist.get_world_size() > 1:
        _calls[0] += 1
        dist.barrier()
        queue = StoreQueue(len(xys), '%d.%d' % (_calls[0], len(xys)))
        rank = dist.get_rank()
    else:
        queue = LocalQueue(len(xys))
        rank = 0
    if device is None:
        import os
        device = int(os.environ.get('LOCAL_RANK', '0'))
    log.info('change detection of %d chips, %d per launch, rank %d' % (len(xys), batch_chips, rank))
    sink, stats = detect_tile(xys, source, queue, device=device, contexts=contexts, batch_chips=batch_chips,
                              params=params, width=width, sink=sink, context_factory=context_factory,
                              upload_depth=upload_depth)
    stats['rank'] = rank
    chip_summaries = getattr(sink, 'chips', [])
    parts = gather((stats, chip_summaries), dist if dist_on else None)
    if parts is None:
        return None
    summaries = sorted((s for _, cs in parts for s in cs), key=lambda s: s['pos'])
    done = [s['pos'] for s in summaries]
    if done != list(range(len(xys))):
        raise RuntimeError('tile incomplete: %d of %d chips processed' % (len(set(done)), len(xys)))
    return {'xys': tuple(xys[p] for p in done), 'chips': summaries, 'ranks': [st for st, _ in parts]}
