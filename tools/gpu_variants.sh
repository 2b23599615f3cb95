#!/bin/bash
# GPU tests with the default kernel, then bench across kernel variants (developer tool).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG=${1:-var}
timeout -k 10 900 python -m pytest tests -m gpu -x -q > "$OUT/${TAG}_pytest_gpu.log" 2>&1 || { echo "rc=$?" > "$OUT/${TAG}_rc.txt"; exit 1; }
for v in "w4 16" "w4 8" "w1 4"; do
  set -- $v
  CCDGPU_KERNEL=$1 CCDGPU_SLOTS_PER_CU=$2 timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline > "$OUT/${TAG}_bench_$1_$2.json" 2> "$OUT/${TAG}_bench_$1_$2.err" || { echo "rc=$? at $v" > "$OUT/${TAG}_rc.txt"; exit 1; }
done
echo "rc=0" > "$OUT/${TAG}_rc.txt"
