#!/bin/bash
# A/B of detection-library builds on the GPU box (developer tool): GPU parity tests of the default
# build, then golden parity + a short C3 bench of each library named in LIBS (lib/<name>.so).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG=${1:-ab}
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "golden or chip_vs_oracle or param_variants" > "$OUT/${TAG}_pytest.log" 2>&1 || { echo "rc=$? tests" > "$OUT/${TAG}_rc.txt"; exit 1; }
for name in ${LIBS:-libccdgpu}; do
  export CCDGPU_LIBRARY="$R/lcmap-firebird_amd/lib/$name.so"
  timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "golden" > "$OUT/${TAG}_${name}_golden.log" 2>&1 || { echo "rc=$? golden $name" > "$OUT/${TAG}_rc.txt"; exit 1; }
  timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-stream --no-packer ${BENCH_ARGS} > "$OUT/${TAG}_${name}.json" 2> "$OUT/${TAG}_${name}.err" || { echo "rc=$? bench $name" > "$OUT/${TAG}_rc.txt"; exit 1; }
done
echo rc=0 > "$OUT/${TAG}_rc.txt"
