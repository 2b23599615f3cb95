#!/bin/bash
# Round-2: instruction-cache counters of the detection kernel (list the SQC counters first).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG=${1:-ic}
export CCD_BENCH_CACHE=/tmp/ccd_bench_cache
CMD="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-tile --no-stream --no-packer --contexts 1"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 -L > "$OUT/${TAG}_counters.txt" 2>&1 || echo "list rc=$?"
grep -oE "SQC_[A-Z0-9_]+|SQ_IFETCH[A-Z0-9_]*|SQ_INST_LEVEL[A-Z0-9_]*|SQ_WAIT_INST[A-Z0-9_]*" "$OUT/${TAG}_counters.txt" | sort -u > "$OUT/${TAG}_sqc.txt"
cat "$OUT/${TAG}_sqc.txt" | tr '\n' ' '; echo
i=0
for set in "${@:2}"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$OUT/${TAG}pmc_p$i" -o run -- $CMD > "$OUT/${TAG}pmc_p$i.log" 2>&1 || { echo "pmc rc=$? pass $i"; exit 1; }
done
echo done
