#!/bin/bash
# Single-context rocprofv3 kernel-stats pass of the resident leg (the average dispatch duration is
# the per-launch duration behind bench.py's roofline) and, with PMC=1, the PMC passes of
# tools/gpu_pmc.sh (summarised on the CPU by tools/pmc_summary.py --write).  Usage: TAG
set -o pipefail
TAG=${1:-ev}
R=$(pwd); O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats -o run -- python3 $R/bench.py --no-tile --no-packer --no-cpu-baseline --contexts 1 --steps 6 --warmup 1 --roofline-launches 3 > $O/stats_bench.json 2> $O/stats_bench.err || { echo "stats rc=$?"; tail -5 $O/stats_bench.err; exit 1; }
cd $R
python3 tools/rocpd_stats.py $O/stats/run_results.db $O/kernel_stats.csv && head -4 $O/kernel_stats.csv
python3 -c "import json; d=json.load(open('$O/stats_bench.json')); r=d['roofline']; print('stats run: frac', round(r['frac'],4), 'launch_ms', round(r['kernel_ms_per_launch'],2), r['kernel_ms_single_context_launches'])"
rm -f $O/stats/run_results.db
if [ "${PMC:-0}" = 1 ]; then
  bash tools/gpu_pmc.sh ${TAG}_pmc || { echo "pmc failed"; cat gpurun_out/${TAG}_pmc_rc.txt; exit 1; }
  echo pmc ok
fi
