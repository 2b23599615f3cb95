#!/bin/bash
# The other synthetic tile configs through bench.py at HEAD (developer tool): C2 (sparse cadence),
# C4 (mixed QA: snow / insufficient-clear pixels), C5 (change-dense), each on its own tile's
# chip mix.  Each leg has its own time limit; the first failure ends the session.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG=${1:-cfg}
B="python bench.py --steps 3 --no-cpu-baseline --no-stream --no-packer --no-tile"
run() { local name=$1; shift; timeout -k 10 300 $B "$@" > "$OUT/${TAG}_$name.json" 2> "$OUT/${TAG}_$name.err" || { echo "rc=$? $name" > "$OUT/${TAG}_rc.txt"; exit 1; }; }
run c2 --config 2 && run c4 --config 4 && run c5 --config 5
rc=$?; echo "rc=$rc" > "$OUT/${TAG}_rc.txt"; exit $rc
