#!/bin/bash
# Round-2: PCIe probe + bench on the tile mix (no CPU baseline).  Run via gpurun.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/h2d_probe.py > gpurun_out/h2d.json 2> gpurun_out/h2d.err || { echo "probe rc=$?"; tail -20 gpurun_out/h2d.err; exit 1; }
cat gpurun_out/h2d.json
timeout -k 10 900 python -u bench.py --steps 4 --no-cpu-baseline --no-packer > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
