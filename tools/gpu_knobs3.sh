#!/bin/bash
# Knob sweep on the GPU box: chips per launch x contexts per GPU (developer tool).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG=${1:-knobs3}
B="python bench.py --steps 3 --no-cpu-baseline --no-stream --no-packer"
run() { local name=$1; shift; timeout -k 10 300 $B "$@" > "$OUT/${TAG}_$name.json" 2> "$OUT/${TAG}_$name.err" || { echo "rc=$? $name" > "$OUT/${TAG}_rc.txt"; exit 1; }; }
run c64x2 --chips 64 --contexts 2 && run c96x2 --chips 96 --contexts 2 && run c128x2 --chips 128 --contexts 2 && \
run c64x3 --chips 64 --contexts 3 && run c128x1 --chips 128 --contexts 1
rc=$?; echo "rc=$rc" > "$OUT/${TAG}_rc.txt"; exit $rc
