#!/bin/bash
# Round-2: two-rank rehearsal on one GPU (shared device, gloo, tile leg with the shared queue),
# then the default bench line with both CPU baselines.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export CCD_BENCH_CACHE=/tmp/ccd_bench_cache
SECONDS=0; timeout -k 10 1200 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench_full.err; exit 1; }
cat gpurun_out/bench_full.json
echo "bench wall seconds: $SECONDS"
