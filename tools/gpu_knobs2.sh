#!/bin/bash
# Knob sweep (developer tool): resident waves per CU and the w4 register budget, C3 bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG=${1:-k2}
B="python bench.py --steps 3 --no-cpu-baseline --no-stream --no-packer"
run() { local name=$1; shift; env "$@" timeout -k 10 300 $B > "$OUT/${TAG}_$name.json" 2> "$OUT/${TAG}_$name.err" || { echo "rc=$? $name" > "$OUT/${TAG}_rc.txt"; exit 1; }; }
run s10 CCDGPU_SLOTS_PER_CU=10
run s11 CCDGPU_SLOTS_PER_CU=11
run w4 CCDGPU_KERNEL=w4
run base CCDGPU_KERNEL=w3
echo rc=0 > "$OUT/${TAG}_rc.txt"
