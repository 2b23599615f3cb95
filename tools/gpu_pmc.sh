#!/bin/bash
# rocprofv3 PMC passes over one short bench run (separate passes; kernel-trace only, no sys-trace).
# Each pass is SIGKILL-bounded: a counter request the hardware cannot hold hangs rocprofv3.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG=${1:-pmc}
CMD="python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-packer --no-tile --chips ${CHIPS:-64} --contexts 1 --config ${CONFIG:-3}"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$OUT/${TAG}_p$i" -o run -- $CMD > "$OUT/${TAG}_p$i.log" 2>&1 || { echo "rc=$? pass $i" > "$OUT/${TAG}_rc.txt"; exit 1; }
done
echo rc=0 > "$OUT/${TAG}_rc.txt"
