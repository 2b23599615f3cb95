#!/bin/bash
# GPU tests, phase profile (C3, C5) and a short bench (developer loop).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG=${1:-qc}
timeout -k 10 900 python -m pytest tests -m gpu -x -q > "$OUT/${TAG}_pytest_gpu.log" 2>&1 || { echo "rc=$? tests" > "$OUT/${TAG}_rc.txt"; exit 1; }
timeout -k 10 200 python tools/phase_profile.py 3 2 > "$OUT/${TAG}_phase3.json" 2>&1 || { echo "rc=$? phase3" > "$OUT/${TAG}_rc.txt"; exit 1; }
timeout -k 10 200 python tools/phase_profile.py 5 1 > "$OUT/${TAG}_phase5.json" 2>&1 || { echo "rc=$? phase5" > "$OUT/${TAG}_rc.txt"; exit 1; }
timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err" || { echo "rc=$? bench" > "$OUT/${TAG}_rc.txt"; exit 1; }
echo "rc=0" > "$OUT/${TAG}_rc.txt"
# A/B: the LDS-period build (w1) on the same bench
CCDGPU_LIBRARY="$R/lcmap-firebird_amd/lib/libccdgpu_lds.so" timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline > "$OUT/${TAG}_bench_lds.json" 2> "$OUT/${TAG}_bench_lds.err" || { echo "rc=$? bench_lds" >> "$OUT/${TAG}_rc.txt"; exit 1; }
