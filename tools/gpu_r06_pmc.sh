#!/bin/bash
# Round-6 profiles at HEAD (developer tool, GPU box): the single-context rocprofv3 kernel-stats pass
# of the C3 resident leg and its PMC passes (STATS=1), or the PMC passes of the other configs'
# 16-chip resident legs (CONFIGS="2 4 5"), each summarised on the CPU afterwards by
# tools/pmc_summary.py --write.  Every rocprofv3 run is bounded (tools/gpu_pmc.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
if [ "${STATS:-0}" = 1 ]; then
  PMC=1 bash tools/gpu_evidence_stats.sh r06_stats || { echo "stats failed"; exit 1; }
fi
for c in ${CONFIGS:-}; do
  CONFIG=$c CHIPS=16 bash tools/gpu_pmc.sh r06_c${c}_pmc || { echo "c$c pmc failed"; cat gpurun_out/r06_c${c}_pmc_rc.txt; exit 1; }
  echo "c$c pmc ok"
done
