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

    def remaining(self):
        with self._lock:
            return self.total - self._next


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

    def remaining(self):
        return max(0, self.total - int(self.store.add(self.key, 0)))


# --------------------------------------------------------------------------- host placement
def node_cpus(node):
    """CPU ids of NUMA node ``node`` (sysfs cpulist), or None."""
    try:
        text = open('/sys/devices/system/node/node%d/cpulist' % int(node)).read().strip()
    except (OSError, ValueError):
        return None
    cpus = set()
    for part in text.split(','):
        if '-' in part:
            a, b = part.split('-')
            cpus.update(range(int(a), int(b) + 1))
        elif part:
            cpus.add(int(part))
    return cpus


def bind_to_device_node(device, numa_node=None):
    """Restrict the calling thread -- and every thread it starts afterwards (worker, fetch and
    copy threads inherit it) -- to the CPUs of the NUMA node GPU ``device`` is attached to,
    within the current affinity, so the host copies of chip data and the pinned buffers they
    land in (first touched by those threads) sit on the socket the GPU's DMA reads from.
    Returns the previous affinity (for restore_affinity), or None when the node is unknown or
    the intersection is empty (nothing changed)."""
    import os
    if not hasattr(os, 'sched_getaffinity'):
        return None
    if numa_node is None:
        try:
            import ccdgpu
            numa_node = ccdgpu.device_numa_node(device)
        except Exception:  # no GPU runtime / device here: leave the placement alone
            return None
    if numa_node is None or numa_node < 0:
        return None
    cpus = node_cpus(numa_node)
    old = os.sched_getaffinity(0)
    want = (cpus or set()) & old
    if not want or want == old:
        return None
    os.sched_setaffinity(0, want)
    return old


def restore_affinity(old):
    import os
    if old:
        os.sched_setaffinity(0, old)


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
    ccdc.sink) as <directory>/<table>/<cx>_<cy>.parquet, plus a SummarySink record.

    Parquet encoding costs ~0.7 s of one core per C3 chip (the pixel table's n_pix x n_obs mask
    entries), far more than its detection: ``threads`` > 0 writes on a pool of
    that many threads (pyarrow encodes without the GIL) from copies of the chip's arrays, so
    the runner's workers hand a chip over and go back to the device -- at most ``max_pending``
    chips (default 2 x threads) wait for a writer, beyond that the handing worker blocks, so the
    copies held for the pool stay bounded when the writers are slower than the device (they are:
    ~12 chips/s against ~330).  ``flush()`` waits for the writes and raises the first write error;
    the tile driver calls it before it returns.
    ``options``: pyarrow.parquet.write_table options for every file.  Measured on one MI355X box
    (16 CPUs, `tools/parquet_tile.py`, 96 chips): 7.6 chips/s inline, 10.9 / 11.9 with 8 / 14
    writer threads -- the box's CPUs, not the device, bound a tile written this way."""

    def __init__(self, directory, threads=0, max_pending=None, **options):
        self.directory = directory
        self.options = options  # pyarrow.parquet.write_table options (ccdc.sink.write_parquet)
        self.summary = SummarySink()
        self._pool = None
        self._pending = []
        self._lock = threading.Lock()
        self._slots = None
        if int(threads) > 0:
            from concurrent.futures import ThreadPoolExecutor
            self._pool = ThreadPoolExecutor(int(threads), thread_name_prefix='ccd-parquet')
            n = int(max_pending) if max_pending is not None else 2 * int(threads)
            if n < 1:
                raise ValueError('max_pending must be >= 1, got %d' % n)
            self._slots = threading.BoundedSemaphore(n)

    def _write(self, cx, cy, dates, row_offsets, rows, mask_bits):
        from ccdc import sink
        from ccdgpu import abi
        mask = abi.unpack_mask_bits(mask_bits, dates.shape[0])
        sink.write_parquet(self.directory, sink.tables(cx, cy, dates, row_offsets, rows, mask), cx, cy,
                           **self.options)

    def __call__(self, pos, cx, cy, dates, row_offsets, rows, mask_bits):
        if self._pool is None:
            self._write(cx, cy, dates, row_offsets, rows, mask_bits)
        else:
            # the runner's arrays are views of reused landing buffers: copies go to the pool
            self._slots.acquire()  # backpressure: at most max_pending chips queued or being written
            try:
                f = self._pool.submit(self._write, cx, cy, np.array(dates), np.array(row_offsets), np.array(rows),
                                      np.array(mask_bits))
            except BaseException:
                self._slots.release()
                raise
            f.add_done_callback(lambda _f: self._slots.release())
            with self._lock:
                self._pending.append(f)
        self.summary(pos, cx, cy, dates, row_offsets, rows, mask_bits)

    def flush(self):
        """Wait for every submitted write; raise the first failure."""
        with self._lock:
            pending, self._pending = self._pending, []
        first = None
        for f in pending:
            e = f.exception()
            if e is not None and first is None:
                first = e
        if first is not None:
            raise first

    def close(self):
        try:
            self.flush()
        finally:
            if self._pool is not None:
                self._pool.shutdown(wait=True)
                self._pool = None

    @property
    def chips(self):
        return self.summary.chips


# --------------------------------------------------------------------------- transport encoding
class EncodingSource(object):
    """Source wrapper for the upload: every batch the wrapped ``source`` returns is encoded into a
    pinned ``ccdgpu.EncodedBatch`` by ``threads`` host threads in the fetch thread, and decoded on
    the device after the upload (include/ccdgpu.h, ccd_encode.c).  ``drop='unread'`` (default):
    observations whose QA word has the fill, cloud or shadow bit send no band values -- no pyccd
    procedure keeps those classes, so the detection never reads them and its results are the
    same (``ccdgpu.unread_drop_bits(params)``); ``drop='lossless'``: only fill observations
    holding -9999, so the device inputs equal the raw ones bit for bit.  QA words travel as 4-bit
    palette codes either way; chips that do not fit go raw.  On the tile mix 'unread' sends ~47 %
    of the raw bytes, 'lossless' ~82 %: the PCIe link bounds the tile.  The encode
    is the pass every fetched chip needs anyway to reach pinned memory: a source with a
    ``views(positions)`` method hands over its own arrays (no copy before the encode); otherwise
    its batch is encoded and released at once.  ``bytes_raw`` / ``bytes_sent`` count the traffic."""

    def __init__(self, source, threads=4, pinned=None, drop='unread', params=None):
        import ccdgpu
        self.source = source
        self.threads = int(threads)
        if drop == 'unread':
            self.drop_bits, self.strict_bits = ccdgpu.unread_drop_bits(params)
        elif drop == 'lossless':
            self.drop_bits = self.strict_bits = 1
        else:
            raise ValueError("drop must be 'unread' or 'lossless', got %r" % (drop,))
        self.drop = drop
        self.pinned = pinned  # None: pinned when the runtime can page-lock (a GPU host), else pageable
        self._free = []
        self._lock = threading.Lock()
        self.bytes_raw = 0
        self.bytes_sent = 0
        self.encode_seconds = 0.0

    def __call__(self, positions):
        import ccdgpu
        t0 = time.perf_counter()
        views = getattr(self.source, 'views', None) if getattr(self.source, 'has_views', True) else None
        raw = None
        if views is not None:
            chips = views(positions)
        else:
            raw = self.source(positions)
            chips = [raw.chip(c) for c in range(raw.n_chips)]
        n_pix = [int(c[2].shape[0]) for c in chips]
        n_obs = [int(c[0].shape[0]) for c in chips]
        need = len(chips), max(n_pix), max(n_obs)
        st = None
        with self._lock:
            for i, (shape, cand) in enumerate(self._free):
                if shape[0] >= need[0] and shape[1] >= need[1] and shape[2] >= need[2]:
                    st = self._free.pop(i)
                    break
        if st is None:
            st = (need, self._storage(need))
        b = ccdgpu.EncodedBatch(n_pix, n_obs, storage=st[1])
        b._enc_storage = st
        b.fill(chips, self.threads, self.drop_bits, self.strict_bits)
        if raw is not None:
            release = getattr(self.source, 'release', None)
            if release is not None:
                release(raw)  # encoded: the raw batch's buffers are free again
        with self._lock:
            self.bytes_raw += sum(16 * p * o + 8 * o for p, o in zip(n_pix, n_obs))
            self.bytes_sent += b.nbytes_encoded + b.dates.nbytes
            self.encode_seconds += time.perf_counter() - t0
        return b

    def _storage(self, need):
        import ccdgpu
        if self.pinned is not False:
            try:
                return ccdgpu.encode_storage(*need, pinned=True)
            except ccdgpu.CcdGpuError:
                if self.pinned:
                    raise
                self.pinned = False  # no device runtime here: pageable buffers (synchronous uploads)
        return ccdgpu.encode_storage(*need, pinned=False)

    def release(self, batch):
        st = getattr(batch, '_enc_storage', None)
        if st is not None:
            with self._lock:
                self._free.append(st)

    def prefill(self, n, n_chips, max_pix, max_obs):
        """Allocate ``n`` encoded-batch buffers ahead (page-locking is slow: outside a timed run)."""
        for _ in range(int(n)):
            need = (int(n_chips), int(max_pix), int(max_obs))
            st = self._storage(need)
            with self._lock:
                self._free.append((need, st))

    def close(self):
        """Drop the free encoded-batch buffers (their pinned memory is released with the last
        view); batches still handed out keep theirs."""
        with self._lock:
            self._free = []


# --------------------------------------------------------------------------- the GPU worker
def _pull_size(queue, batch_chips, tail_chips):
    """Chips to take next: a full batch, or a quarter batch once fewer than ``tail_chips``
    positions remain, so the last chips of a tile spread over every worker of every rank
    instead of waiting in one worker's upload queue."""
    if tail_chips and batch_chips > 1 and hasattr(queue, 'remaining') and queue.remaining() < tail_chips:
        return max(1, batch_chips // 4)
    return batch_chips


def _fetcher(queue, source, batch_chips, tail_chips, stats, ready, stop, permits):
    """A worker's fetch thread: pulls the next positions from the shared queue and asks the source
    for their ARD (the merlin / chipmunk fetch stand-in; often I/O- or copy-bound), so the fetch
    of the next batches overlaps the upload, detection and row fetch of the current ones.  Puts
    (positions, batch) on ``ready``, then None when the queue is empty, or the exception that
    stopped it.  A fetch starts only with one of the worker's upload-slot ``permits`` (a slot
    that is free or will be by the time the batch arrives), so at most depth + 1 batches of a
    worker are fetched or staged at once -- the source's buffers stay bounded."""
    clock = time.perf_counter
    try:
        while not stop.is_set():
            if not permits.acquire(timeout=0.1):
                continue
            t0 = clock()
            pos = queue.next(_pull_size(queue, batch_chips, tail_chips))
            if not pos:
                with stats['lock']:
                    stats['queue_empty_at'] = max(stats['queue_empty_at'], t0 - stats['t0'])
                ready.put(None)
                return
            batch = source(pos)
            if batch.n_chips != len(pos):
                raise ValueError('source returned %d chips for %d positions' % (batch.n_chips, len(pos)))
            with stats['lock']:
                stats['source_seconds'] += clock() - t0
            ready.put((pos, batch))
    except BaseException as e:
        ready.put(e)


def _worker(ctx, queue, source, xys, batch_chips, params, width, sink, stats, errors, depth=2, tail_chips=0):
    """One context: up to ``depth`` batches uploaded (or uploading) ahead of the one being
    detected, one upload slot each, so the PCIe link stays busy while a batch is detected and
    its rows are fetched (with one batch ahead the link idles whenever both of a GPU's contexts
    are past their upload).  The ARD of the next batches is fetched by the worker's own fetch
    thread (``_fetcher``) meanwhile.  Near the end of the queue the batches shrink (``_pull_size``)."""
    import os
    import queue as queue_mod
    # CCDC_RUNNER_TRACE=1: per-batch host timestamps (perf_counter) of this worker into
    # stats['trace'] -- staged / launched / detection done / rows fetched (diagnostics)
    trace = [] if os.environ.get('CCDC_RUNNER_TRACE') else None
    ready = queue_mod.Queue()
    stop = threading.Event()
    permits = threading.Semaphore(depth + 1)  # one per upload slot
    ft = threading.Thread(target=_fetcher, args=(queue, source, batch_chips, tail_chips, stats, ready, stop, permits),
                          daemon=True, name='ccd-fetch-%s' % threading.current_thread().name.rsplit('-', 1)[-1])
    ft.start()
    try:
        clock = time.perf_counter
        free = list(range(depth + 1))
        staged = []  # (slot, positions, batch), in upload order
        split = hasattr(ctx, 'run_slot_begin')  # (test doubles have run_slot only)
        into = None  # the context's reusable pinned landing buffers for the rows
        if hasattr(ctx, 'fetch_batch_rows_into'):
            import ccdgpu
            into = ccdgpu.RowsBuffers()
        # the rows come back in the detection's own device chain (one wait per batch instead of
        # a wait for the detection and then the CSR, row packing and copies with their own waits)
        chain = into is not None and hasattr(ctx, 'run_slot_begin_rows') and not os.environ.get('CCDC_NO_ROW_CHAIN')
        exhausted = False
        while True:
            while free and not exhausted:
                # with a batch staged, upload only what is already fetched; otherwise wait for it
                try:
                    item = ready.get(block=not staged)
                except queue_mod.Empty:
                    break
                if item is None:
                    exhausted = True
                    break
                if isinstance(item, BaseException):
                    raise item
                pos, batch = item
                t1 = clock()
                slot = free.pop(0)
                ctx.stage_slot_chips(slot, batch, params)
                staged.append((slot, pos, batch))
                if trace is not None:
                    trace.append(('stage', pos[0], t1))
                with stats['lock']:
                    stats['stage_seconds'] += clock() - t1
            if not staged:
                break
            s, ppos, pbatch = staged.pop(0)
            cx = np.array([xys[p][0] for p in ppos], dtype=np.int32)
            cy = np.array([xys[p][1] for p in ppos], dtype=np.int32)
            t2 = clock()
            t_in = 0.0  # staging done while the detection ran
            got = None
            if split:
                if chain:
                    ctx.run_slot_begin_rows(s, cx, cy, into, width)
                else:
                    ctx.run_slot_begin(s)
                # while it runs, upload what the fetch thread finishes into the free slots (a
                # batch otherwise waits for this detection and its row fetch to end)
                while free and not exhausted and not ctx.run_done():
                    try:
                        item = ready.get(timeout=0.002)
                    except queue_mod.Empty:
                        continue
                    if item is None:
                        exhausted = True
                        break
                    if isinstance(item, BaseException):
                        raise item
                    pos, batch = item
                    t1 = clock()
                    slot = free.pop(0)
                    ctx.stage_slot_chips(slot, batch, params)
                    staged.append((slot, pos, batch))
                    if trace is not None:
                        trace.append(('stage', pos[0], t1))
                    t_in += clock() - t1
                t_end = clock()
                if chain:
                    got = ctx.run_slot_end_rows()
                else:
                    ctx.run_slot_end()
            else:
                t_end = clock()
                ctx.run_slot(s)
            if getattr(ctx, 'qa_error', False):
                import ccdgpu
                raise ccdgpu.QAValueError('unsupported bit-packed QA value in chips at tile positions %s' % (ppos,))
            t3 = clock()
            if got is not None:  # views of the landing buffers: valid until the next batch
                off, rows, mask = got
            elif into is not None:  # views of the landing buffers: valid until the next batch's fetch
                off, rows, mask = ctx.fetch_batch_rows_into(cx, cy, into, width)
            else:
                off, rows, mask = ctx.fetch_batch_rows(cx, cy, width)
            free.append(s)  # its rows are fetched: the slot takes the next upload
            permits.release()
            t4 = clock()
            for c, p in enumerate(ppos):
                p0, p1 = int(pbatch.pix_off[c]), int(pbatch.pix_off[c + 1])
                r0, r1 = int(off[p0]), int(off[p1])
                d, _, _ = pbatch.chip(c)
                sink(p, int(cx[c]), int(cy[c]), d, off[p0:p1 + 1] - r0, rows[r0:r1], pbatch.mask_bits_of(mask, c))
            release = getattr(source, 'release', None)
            if release is not None:
                release(pbatch)  # its upload is done and its rows are out: the source may reuse it
            t5 = clock()
            if trace is not None:
                # launch, (begin of) the wait for the detection, detection finished, rows fetched, sunk
                trace.append(('run', ppos[0], t2, t_end, t3, t4, t5))
            with stats['lock']:
                stats['batches'] += 1
                stats['chips'] += len(ppos)
                stats['pixels'] += pbatch.total_pixels
                stats['rows'] += int(rows.shape[0])
                stats['device_seconds'] += t3 - t2 - t_in
                stats['stage_seconds'] += t_in
                stats['fetch_seconds'] += t4 - t3
                stats['sink_seconds'] += t5 - t4
    except BaseException as e:  # reported by detect_tile after the other workers drain
        errors.append(e)
    finally:
        if trace is not None:
            with stats['lock']:
                stats.setdefault('trace', []).append([(x[0], x[1]) + tuple(round(v - stats['t0'], 5) for v in x[2:])
                                                      for x in trace])
        stop.set()
        while ft.is_alive():  # unblock a fetcher waiting to put (its batch is dropped)
            try:
                ready.get(timeout=0.05)
            except queue_mod.Empty:
                pass
        ft.join()


def detect_tile(xys, source, queue, device=0, contexts=4, batch_chips=6, params=None, width=100,
                sink=None, context_factory=None, upload_depth=2, tail_chips=None, bind_numa=True, encode=True,
                encode_threads=3, copy_cus=8):
    """Change detection of the tile chips at ``xys`` (list of (cx, cy), tile order) on one GPU.

    ``source(positions) -> ccdgpu.ChipBatch`` supplies the ARD of the chips at those tile
    positions (pinned batches upload asynchronously; a source with a ``release(batch)`` method
    gets each batch back once its rows are fetched, to reuse its buffers); ``queue`` hands out positions (LocalQueue
    for one process, StoreQueue across ranks); ``sink(pos, cx, cy, dates, row_offsets, rows,
    mask_bits)`` receives each chip's device-packed rows and its processing masks as bit words
    [n_pix][words] (ccdgpu.abi.unpack_mask_bits; default sink: a SummarySink) -- views of the
    context's reusable landing buffers, valid during the call: a sink that keeps them copies.  Returns the sink
    and this process's statistics.  ``upload_depth``: batches each context keeps uploaded or
    uploading ahead of the one it detects (1 .. ccdgpu.UPLOAD_SLOTS - 1).  ``tail_chips``: once
    fewer positions than this remain in the queue, workers pull quarter batches (default: two
    full batches per context of this process).  ``encode``: upload every batch in the transport
    encoding (EncodingSource, ``encode_threads`` host threads per fetch; True = its 'unread'
    setting, 'lossless' = lossless) instead of raw -- ``source`` may then also be an
    EncodingSource already (its counters are reported).  ``copy_cus``: CUs each context reserves
    for its upload (decode kernel, blits) so other contexts' persistent detection waves cannot
    starve it (ccdgpu_init_copy_cus; 0 = none; not used with a ``context_factory``)."""
    from ccdgpu import UPLOAD_SLOTS
    if not 1 <= int(upload_depth) <= UPLOAD_SLOTS - 1:
        raise ValueError('upload_depth must be in 1 .. %d (ccdgpu.UPLOAD_SLOTS - 1), got %r' % (UPLOAD_SLOTS - 1, upload_depth))
    if int(batch_chips) < 1:
        raise ValueError('batch_chips must be >= 1, got %r' % (batch_chips,))
    if tail_chips is None:
        tail_chips = 2 * int(batch_chips) * max(1, int(contexts))
    if context_factory is None:
        import ccdgpu

        def context_factory(dev):
            return ccdgpu.Context(dev, copy_cus=copy_cus)
    if encode and not isinstance(source, EncodingSource):
        source = EncodingSource(source, threads=encode_threads, drop='lossless' if encode == 'lossless' else 'unread',
                                params=params)
    sink = sink if sink is not None else SummarySink()
    # per-phase host seconds summed over the workers: source (ARD fetch), stage (upload call),
    # device (run_slot: waits for the upload, detects), fetch (row packing + D2H), sink
    # queue_empty_at: seconds from the start until a worker first found the queue empty (the
    # rest of this process's time is its tail: the last batches draining)
    t0 = time.perf_counter()
    stats = {'lock': threading.Lock(), 't0': t0, 'batches': 0, 'chips': 0, 'pixels': 0, 'rows': 0, 'device_seconds': 0.0,
             'source_seconds': 0.0, 'stage_seconds': 0.0, 'fetch_seconds': 0.0, 'sink_seconds': 0.0,
             'queue_empty_at': 0.0}
    errors = []
    ctxs = [context_factory(device) for _ in range(max(1, int(contexts)))]
    # worker / fetch / copy threads on the GPU's NUMA node (restored when the tile is done)
    old_aff = bind_to_device_node(device) if bind_numa else None
    try:
        th = [threading.Thread(target=_worker, args=(c, queue, source, xys, int(batch_chips), params, width, sink, stats,
                                                       errors, int(upload_depth), int(tail_chips)), name='ccd-worker-%d' % i)
              for i, c in enumerate(ctxs)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        flush = getattr(sink, 'flush', None)
        if flush is not None:
            try:
                flush()  # a sink that writes in the background (ParquetSink(threads=...)) is done
            except BaseException as e:
                errors.append(e)
    finally:
        for c in ctxs:
            c.close()
        restore_affinity(old_aff)
    stats.pop('lock')
    stats.pop('t0')
    stats['seconds'] = time.perf_counter() - t0
    if isinstance(source, EncodingSource):
        stats['upload_bytes_raw'] = source.bytes_raw
        stats['upload_bytes_sent'] = source.bytes_sent
        stats['encode_seconds'] = source.encode_seconds
    stats['tail_seconds'] = stats['seconds'] - stats['queue_empty_at'] if stats['queue_empty_at'] else 0.0
    if errors:
        errors[0].tile_stats = stats  # what this process did before the failure (changedetection's gather)
        raise errors[0]
    return sink, stats


_calls = [0]
_gloo = {}  # one gloo group per default process group (created once, reused by every gather)


def gather(obj, dist=None):
    """All ranks' ``obj`` as a list on rank 0 (None elsewhere); [obj] without a process group.
    Uses a gloo group (created on first use and cached), so it works whatever backend the
    default group has."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return [obj]
    from torch.distributed import distributed_c10d
    key = id(distributed_c10d._get_default_group())
    group = _gloo.get(key)
    if group is None:
        _gloo.clear()  # a group of an earlier (destroyed) default group is stale
        group = _gloo[key] = dist.new_group(backend='gloo')
    out = [None] * dist.get_world_size() if dist.get_rank() == 0 else None
    dist.gather_object(obj, out, dst=0, group=group)
    return out


class TileError(RuntimeError):
    """A rank's worker failed during changedetection: raised on every rank after the gather, on
    rank 0 with the first failing rank's error (``rank``, ``cause``)."""

    def __init__(self, rank, cause):
        super(TileError, self).__init__('rank %d: %s: %s' % (rank, type(cause).__name__, cause))
        self.rank = rank
        self.cause = cause


def changedetection(tile, source, device=None, contexts=4, batch_chips=6, number=None, params=None,
                    sink=None, width=100, context_factory=None, ctx=None, upload_depth=2, tail_chips=None,
                    bind_numa=True, encode=True, encode_threads=3, copy_cus=8):
    """Change detection for a tile on every GPU of the job (reference core.changedetection,
    ccdc/core.py:78-123).

    ``tile``: {'chips': [[cx, cy], ...]} (grid.tile's response, test/data/tile_response.json) or
    a plain list of (cx, cy); ``number`` limits the chips (the reference's testing knob);
    ``source(positions) -> ChipBatch``.  Under torch.distributed every rank calls this with the
    same arguments: ranks share one dynamic chip queue and rank 0 gets the gathered result.
    Returns (on rank 0, else None) {'xys': processed chip coordinates in tile order, 'chips':
    per-chip summaries, 'ranks': per-rank statistics}.

    A worker failure (QA error, device error, a failing source) does not strand the other
    ranks: the failing rank still takes part in the gather, sending its error, and every rank
    then raises -- rank 0 a ``TileError`` carrying the first failing rank's exception (its
    ``cause``), the others their own error.  Without a process group the error propagates
    unchanged."""
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
    error = None
    try:
        sink, stats = detect_tile(xys, source, queue, device=device, contexts=contexts, batch_chips=batch_chips,
                                  params=params, width=width, sink=sink, context_factory=context_factory,
                                  upload_depth=upload_depth, tail_chips=tail_chips, bind_numa=bind_numa,
                                  encode=encode, encode_threads=encode_threads, copy_cus=copy_cus)
    except Exception as e:
        if not (dist_on and dist.get_world_size() > 1):
            raise
        error = e
        stats = dict(getattr(e, 'tile_stats', {}))
    stats['rank'] = rank
    chip_summaries = getattr(sink, 'chips', []) if error is None else []
    err_msg = None if error is None else (type(error).__name__, str(error))
    parts = gather((stats, chip_summaries, err_msg), dist if dist_on else None)
    if error is not None:
        if rank == 0:
            raise TileError(0, error)
        raise error
    if parts is None:
        return None
    failed = [(st.get('rank', r), e) for r, (st, _, e) in enumerate(parts) if e is not None]
    if failed:
        r, (name, msg) = failed[0]
        raise TileError(r, RuntimeError('%s: %s' % (name, msg)))
    summaries = sorted((s for _, cs, _ in parts for s in cs), key=lambda s: s['pos'])
    done = [s['pos'] for s in summaries]
    if done != list(range(len(xys))):
        raise RuntimeError('tile incomplete: %d of %d chips processed' % (len(set(done)), len(xys)))
    return {'xys': tuple(xys[p] for p in done), 'chips': summaries, 'ranks': [st for st, _, _ in parts]}
