#!/bin/bash
# One kernel variant on the GPU box: its GPU parity tests, then a short bench (developer tool).
#   VARIANT=w4 bash tools/gpu_variant.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG=${1:-var}
export CCDGPU_KERNEL=${VARIANT:-w3}
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "golden or chip_vs_oracle or param_variants" > "$OUT/${TAG}_pytest.log" 2>&1 || { echo "rc=$? tests" > "$OUT/${TAG}_rc.txt"; exit 1; }
timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream --no-packer > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err" || { echo "rc=$? bench" > "$OUT/${TAG}_rc.txt"; exit 1; }
timeout -k 10 300 python bench.py --steps 2 --config 5 --no-cpu-baseline --no-stream --no-packer > "$OUT/${TAG}_bench_c5.json" 2> "$OUT/${TAG}_bench_c5.err" || { echo "rc=$? bench5" > "$OUT/${TAG}_rc.txt"; exit 1; }
echo rc=0 > "$OUT/${TAG}_rc.txt"
