#!/bin/bash
# Developer tool: golden parity + C3 bench for each register-budget variant of the default library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG=${1:-kv}
for kv in ${KERNELS:-w1 w2 w3}; do
  echo -n "$kv " >> "$OUT/${TAG}_parity.log"
  CCDGPU_KERNEL=$kv timeout -k 10 60 python tools/variant_check.py >> "$OUT/${TAG}_parity.log" 2>&1 || { echo "rc=$? parity $kv" >> "$OUT/${TAG}_parity.log"; exit 1; }
  CCDGPU_KERNEL=$kv timeout -k 10 200 python bench.py --steps ${STEPS:-6} --no-cpu-baseline --no-packer --no-stream > "$OUT/${TAG}_bench_$kv.json" 2> "$OUT/${TAG}_bench_$kv.err" || exit 1
done
