#!/bin/bash
# Chip packer profiles (developer tool, GPU box): rocprofv3 kernel stats and the HBM traffic
# passes (FETCH_SIZE, WRITE_SIZE in separate passes) of tools/packer_ab.py, for the form
# selected by CCDGPU_UNPACK_V1 (exported by the caller).  Every pass is SIGKILL-bounded.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG=${1:-pack}
CMD="python3 $R/tools/packer_ab.py"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_stats" -o run -- $CMD > "$OUT/${TAG}_stats.log" 2>&1 || { echo "rc=$? stats"; exit 1; }
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$OUT/${TAG}_p$i" -o run -- $CMD > "$OUT/${TAG}_p$i.log" 2>&1 || { echo "rc=$? pass $i"; exit 1; }
done
echo ok
