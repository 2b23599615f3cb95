#!/usr/bin/env python3
"""Developer tool (GPU box): the tile driver with the offline Parquet sink -- N distinct C3 chips
(bench's pool source, transport-encoded uploads) written as segment / pixel / chip Parquet files,
inline and on writer pools; chips/s of each, beside the summary-only sink.

usage: parquet_tile.py [chips] [outdir]"""
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'lcmap-firebird_amd')]
from ccdc import runner  # noqa: E402
from ccdgpu import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 96
out = sys.argv[2] if len(sys.argv) > 2 else tempfile.mkdtemp(prefix='ccd_parquet_')
src = synth.TileSource(synth.config(3), device=0, batch_chips=6, mode='pool', pool_chips=16, rotate_threads=3)
src.prepare()
xys = [(-1815585 + 3000 * (c // 50), 1064805 - 3000 * (c % 50)) for c in range(n)]
runner.changedetection(xys[:12], src)  # warm
for label, mk in (('summary', lambda: runner.SummarySink(digest=False)),
                  ('parquet inline', lambda: runner.ParquetSink(out)),
                  ('parquet 8 threads', lambda: runner.ParquetSink(out, threads=8)),
                  ('parquet 14 threads', lambda: runner.ParquetSink(out, threads=14))):
    sink = mk()
    t = time.perf_counter()
    runner.changedetection(xys, src, sink=sink)
    el = time.perf_counter() - t
    getattr(sink, 'close', lambda: None)()
    print('%-20s %d chips in %.2f s: %.1f chips/s' % (label, n, el, n / el), flush=True)
    shutil.rmtree(out, ignore_errors=True)
    os.makedirs(out, exist_ok=True)
src.close()
