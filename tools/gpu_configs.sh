#!/bin/bash
# The change-dense C5 tile chips (beside the bench's C3) through bench.py at HEAD (developer tool).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG=${1:-cfg}
B="python bench.py --steps 3 --no-cpu-baseline --no-stream --no-packer"
run() { local name=$1; shift; timeout -k 10 300 $B "$@" > "$OUT/${TAG}_$name.json" 2> "$OUT/${TAG}_$name.err" || { echo "rc=$? $name" > "$OUT/${TAG}_rc.txt"; exit 1; }; }
run c5 --config 5
rc=$?; echo "rc=$rc" > "$OUT/${TAG}_rc.txt"; exit $rc
