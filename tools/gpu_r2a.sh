#!/bin/bash
# Round-2 GPU check: GPU tests, smoke, short bench (no CPU baseline).  Run via gpurun.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 900 python -u bench.py --steps 4 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
