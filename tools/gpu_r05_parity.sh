#!/bin/bash
# Round-5 evidence, second half (GPU box): the C5 PMC passes and the 250k-pixel tile parity run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
T=${TAG:-r05ev}
CONFIG=5 bash tools/gpu_pmc.sh ${T}_c5_pmc || { echo "c5 pmc failed"; cat gpurun_out/${T}_c5_pmc_rc.txt; exit 1; }
echo c5 pmc ok
timeout -k 10 900 python -u tools/tile_parity.py --batch 6 --out gpurun_out/${T}_tile_parity.json > gpurun_out/${T}_tile_parity.log 2>&1 || { echo "parity rc=$?"; tail -20 gpurun_out/${T}_tile_parity.log; exit 1; }
tail -1 gpurun_out/${T}_tile_parity.log
