#!/bin/bash
# Developer loop on the GPU box: gpu tests, short bench (default and LDS-period builds).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG=${1:-loop}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/${TAG}_pytest_gpu.log" 2>&1 || { echo "rc=$? tests" > "$OUT/${TAG}_rc.txt"; exit 1; }
timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err" || { echo "rc=$? bench" > "$OUT/${TAG}_rc.txt"; exit 1; }
timeout -k 10 300 python bench.py --steps 2 --config 5 --no-cpu-baseline > "$OUT/${TAG}_bench_c5.json" 2> "$OUT/${TAG}_bench_c5.err" || { echo "rc=$? bench5" > "$OUT/${TAG}_rc.txt"; exit 1; }
CCDGPU_LIBRARY="$R/lcmap-firebird_amd/lib/libccdgpu_lds.so" timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline > "$OUT/${TAG}_bench_lds.json" 2> "$OUT/${TAG}_bench_lds.err" || { echo "rc=$? bench_lds" > "$OUT/${TAG}_rc.txt"; exit 1; }
echo "rc=0" > "$OUT/${TAG}_rc.txt"
