#!/bin/bash
# Developer tool: instruction/scalar cache PMC pass over one bench step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG=${1:-pmi}
CMD="python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-packer --chips ${CHIPS:-4}"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ SQ_IFETCH SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_ICACHE_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$OUT/${TAG}_p$i" -o run -- $CMD > "$OUT/${TAG}_p$i.log" 2>&1 || { echo "rc=$? pass $i" > "$OUT/${TAG}_rc.txt"; exit 1; }
done
echo rc=0 > "$OUT/${TAG}_rc.txt"
