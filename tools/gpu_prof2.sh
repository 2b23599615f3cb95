#!/bin/bash
# Round-2 profiling session: rocprofv3 kernel-trace stats of the bench's resident leg (one
# context), PMC passes (each its own run, SIGKILL-bounded), phase split of the diag build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG=${1:-r02}
export CCD_BENCH_CACHE=/tmp/ccd_bench_cache
CMD="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-tile --no-stream --no-packer --contexts 1"
# populate the input cache (and a plain reference line) before profiling
timeout -k 10 600 python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-tile --no-stream --no-packer --contexts 1 > "$OUT/${TAG}_plain.json" 2> "$OUT/${TAG}_plain.err" || { echo "plain rc=$?"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof" -o run -- $CMD > "$OUT/${TAG}_prof.log" 2>&1 || { echo "prof rc=$?"; exit 1; }
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$OUT/${TAG}pmc_p$i" -o run -- $CMD > "$OUT/${TAG}pmc_p$i.log" 2>&1 || { echo "pmc rc=$? pass $i"; exit 1; }
done
cd "$R"
timeout -k 10 300 python tools/phase_profile.py 3 2 > "$OUT/${TAG}_phase_c3.json" 2>&1 || { echo "phase rc=$?"; exit 1; }
timeout -k 10 300 python tools/phase_profile.py 5 2 > "$OUT/${TAG}_phase_c5.json" 2>&1 || { echo "phase c5 rc=$?"; exit 1; }
echo done
