#!/bin/bash
# Round-2: tile runner + batch tests on the GPU, then the bench with the tile leg.  Run via gpurun.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_tile.py tests/test_gpu_batches.py tests/test_chipmunk.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_c.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_c.log; exit 1; }
tail -3 gpurun_out/pytest_c.log
timeout -k 10 900 python -u bench.py --steps 4 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
