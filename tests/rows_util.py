"""Host restatement of the device row writer (lcmap-firebird_amd/csrc/ccd_rows.hip) over an
abi.Unpacked result -- test infrastructure for the tile runner's CPU tests (an oracle-backed
stand-in context) and for checking device rows against oracle rows."""
import numpy as np

from ccdgpu import abi


def rows_from_result(u, cx, cy, width=100):
    """abi.Unpacked (one chip) -> (row_offsets [n_pix+1], rows ROW_DTYPE): one row per change
    model, pyccd.default's day-1 row (has_model 0) for a pixel without any; float fields rounded
    to float32 (Spark's FloatType cast)."""
    n_pix = u.n_pix
    counts = np.diff(u.seg_offsets)
    per = np.maximum(counts, 1)
    off = np.concatenate([[0], np.cumsum(per)]).astype(np.int64)
    rows = np.zeros(int(off[-1]), abi.ROW_DTYPE)
    for p in range(n_pix):
        r0 = off[p]
        px, py = cx + 30 * (p % width), cy - 30 * (p // width)
        a, b = int(u.seg_offsets[p]), int(u.seg_offsets[p + 1])
        if b == a:
            rows[r0]['px'], rows[r0]['py'] = px, py
            rows[r0]['sday'] = rows[r0]['eday'] = rows[r0]['bday'] = 1
            continue
        for k, s in enumerate(u.segments[a:b]):
            r = rows[r0 + k]
            r['px'], r['py'] = px, py
            r['sday'], r['eday'], r['bday'] = s['start_day'], s['end_day'], s['break_day']
            r['curqa'], r['has_model'] = s['curve_qa'], 1
            r['chprob'] = np.float32(s['change_probability'])
            r['mag'] = s['magnitude'].astype(np.float32)
            r['rmse'] = s['rmse'].astype(np.float32)
            r['intercept'] = s['intercept'].astype(np.float32)
            r['coef'] = s['coef'].astype(np.float32)
            rows[r0 + k] = r
    return off, rows


def mask_words(mask, words):
    """bool [n_pix][n_obs] -> uint32 [n_pix][words] (bit i of word i/32)."""
    n_pix, n_obs = mask.shape
    bits = np.zeros((n_pix, words * 32), np.uint8)
    bits[:, :n_obs] = mask
    return np.packbits(bits, axis=1, bitorder='little').view('<u4').reshape(n_pix, words)


class OracleContext(object):
    """Stand-in for ccdgpu.Context in CPU tests of the tile runner: the C oracle detects, the
    rows are restated on the host.  Same slot / fetch protocol as the device context."""

    def __init__(self, device=0, threads=2, delay=0.0, fail=None):
        self.device = device
        self.threads = threads
        self.delay = delay
        self.fail = fail  # an exception raised by run_slot (error-path tests of the runner)
        self.qa_error = False
        self._slots = {}
        self._results = None

    def stage_slot_chips(self, slot, batch, params=None):
        import ccdgpu
        if isinstance(batch, ccdgpu.EncodedBatch):  # the runner's transport encoding: decode as the device does
            from encode_util import decode
            chips = decode(batch.buf[:batch.nbytes_encoded])
            batch = ccdgpu.ChipBatch.from_chips([(batch.chip(c)[0], s, q) for c, (s, q) in enumerate(chips)])
        self._slots[slot] = (batch, params)

    def run_slot(self, slot):
        import time
        import oracle_ctypes
        batch, params = self._slots.pop(slot)
        if self.fail is not None:
            raise self.fail
        out = []
        for c in range(batch.n_chips):
            d, s, q = batch.chip(c)
            rc, u = oracle_ctypes.detect_batch(d, s, q, params=params, threads=self.threads)
            self.qa_error = self.qa_error or rc == abi.E_QA
            out.append(u)
        if self.delay:
            time.sleep(self.delay)
        self._results = (batch, out)

    def fetch_batch_rows(self, cx, cy, width=100):
        batch, res = self._results
        words = (int(batch.n_obs.max()) + 31) // 32
        offs, rows, bits = [np.zeros(1, np.int64)], [], []
        for c, u in enumerate(res):
            o, r = rows_from_result(u, int(cx[c]), int(cy[c]), width)
            offs.append(o[1:] + offs[-1][-1])
            rows.append(r)
            bits.append(mask_words(u.mask, words))
        return np.concatenate(offs), np.concatenate(rows), np.concatenate(bits)

    def close(self):
        pass


class SplitOracleContext(OracleContext):
    """OracleContext with the device context's split run (run_slot_begin / run_done /
    run_slot_end): the detection "runs" for ``run_time`` seconds after begin, during which the
    runner stages the batches its fetch thread finishes into other slots."""

    def __init__(self, device=0, threads=2, run_time=0.05, **kw):
        super(SplitOracleContext, self).__init__(device, threads, **kw)
        self.run_time = run_time
        self._pending = None
        self.staged_during_run = 0

    def stage_slot_chips(self, slot, batch, params=None):
        if self._pending is not None:
            assert slot != self._pending[0], 'staged into the slot being detected'
            self.staged_during_run += 1
        super(SplitOracleContext, self).stage_slot_chips(slot, batch, params)

    def run_slot_begin(self, slot):
        import time
        assert self._pending is None, 'run_slot_begin twice'
        assert slot in self._slots, 'slot has no staged batch'
        self._pending = (slot, time.perf_counter() + self.run_time)

    def run_done(self):
        import time
        return self._pending is None or time.perf_counter() >= self._pending[1]

    def run_slot_end(self):
        slot, _ = self._pending
        self._pending = None
        self.run_slot(slot)



class ChainOracleContext(SplitOracleContext):
    """SplitOracleContext with the device context's batch chain (run_slot_begin_rows /
    run_slot_end_rows): the rows land in the caller's RowsBuffers, whose rows room is learned
    from an overflow exactly as ccdgpu.Context does (too small: the rows are fetched after)."""

    def __init__(self, device=0, threads=2, run_time=0.05, **kw):
        super(ChainOracleContext, self).__init__(device, threads, run_time, **kw)
        self.chained = 0
        self.overflowed = 0

    def fetch_batch_rows_into(self, cx, cy, bufs, width=100):
        off, rows, bits = self.fetch_batch_rows(cx, cy, width)
        n_pix, words = bits.shape
        bufs.ensure(off.size, rows.size, bits.size)
        bufs.offsets[:off.size] = off
        bufs.rows[:rows.size] = rows
        bufs.mask[:bits.size] = bits.reshape(-1)
        return bufs.offsets[:off.size], bufs.rows[:rows.size], bufs.mask[:bits.size].reshape(n_pix, words)

    def run_slot_begin_rows(self, slot, cx, cy, bufs, width=100):
        batch = self._slots[slot][0]
        n_pix = int(batch.pix_off[-1])
        words = (int(batch.n_obs.max()) + 31) // 32
        bufs.ensure(n_pix + 1, int(bufs.rows_per_pixel * n_pix) + 64, n_pix * words)
        # the rows the chain copies back: the learned rate, as ccdgpu.Context does
        rate = bufs.copy_per_pixel if bufs.copy_per_pixel is not None else bufs.rows_per_pixel
        cap = min(bufs.rows.size, int(rate * n_pix) + 64)
        self.run_slot_begin(slot)
        self._rows_req = (np.array(cx), np.array(cy), bufs, width, n_pix, cap)

    def run_slot_end_rows(self):
        self.run_slot_end()
        cx, cy, bufs, width, n_pix, cap = self._rows_req
        self.chained += 1
        off, rows, bits = self.fetch_batch_rows(cx, cy, width)
        if rows.size > 0:
            bufs.max_rate = max(bufs.max_rate, rows.size / max(1, n_pix))
            bufs.copy_per_pixel = min(bufs.rows_per_pixel, 1.25 * bufs.max_rate)
        if rows.size > cap:
            self.overflowed += 1
            bufs.rows_per_pixel = max(bufs.rows_per_pixel, 1.25 * rows.size / max(1, n_pix))
            bufs.copy_per_pixel = min(bufs.rows_per_pixel, 1.25 * bufs.max_rate)
        return self.fetch_batch_rows_into(cx, cy, bufs, width)
