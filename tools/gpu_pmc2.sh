#!/bin/bash
# Developer tool: extra rocprofv3 PMC passes (issue mix and memory-pipe stalls) over one bench step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG=${1:-pmx}
CMD="python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-packer --no-stream --chips ${CHIPS:-4}"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD" \
           "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE GRBM_TA_BUSY"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$OUT/${TAG}_p$i" -o run -- $CMD > "$OUT/${TAG}_p$i.log" 2>&1 || { echo "rc=$? pass $i" > "$OUT/${TAG}_rc.txt"; exit 1; }
done
echo rc=0 > "$OUT/${TAG}_rc.txt"
