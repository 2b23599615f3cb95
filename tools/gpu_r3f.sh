#!/bin/bash
# Round-3 GPU call F: rocprofv3 kernel-trace stats of the resident bench, PMC passes (C3 64 chips
# = the bench's resident workload key, C5 32 chips).
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r03f; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats -o run -- python3 $R/bench.py --no-tile --no-packer --no-cpu-baseline --steps 10 --warmup 2 > $O/stats_bench.json 2> $O/stats_bench.err || { echo "stats rc=$?"; exit 1; }
cd $R
TAG=r03f_c3 CONFIG=3 CHIPS=64 bash tools/gpu_pmc.sh r03f_c3 || { echo "pmc c3 failed"; exit 1; }
TAG=r03f_c5 CONFIG=5 CHIPS=32 bash tools/gpu_pmc.sh r03f_c5 || { echo "pmc c5 failed"; exit 1; }
echo done
