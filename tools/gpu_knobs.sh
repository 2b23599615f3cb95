#!/bin/bash
# Knob sweep on the GPU box: chips per launch, kernel register budget (developer tool).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG=${1:-knobs}
B="python bench.py --steps 3 --no-cpu-baseline --no-stream --no-packer"
run() { local name=$1; shift; env "$@" timeout -k 10 300 $B $EXTRA > "$OUT/${TAG}_$name.json" 2> "$OUT/${TAG}_$name.err" || { echo "rc=$? $name" > "$OUT/${TAG}_rc.txt"; exit 1; }; }
EXTRA="--chips 32" run c32 CCDGPU_KERNEL=w3
EXTRA="--chips 64" run c64 CCDGPU_KERNEL=w3
EXTRA="--chips 32" run c32w2 CCDGPU_KERNEL=w2
EXTRA="--chips 32 --config 5" run c5 CCDGPU_KERNEL=w3
echo rc=0 > "$OUT/${TAG}_rc.txt"
