#!/bin/bash
# Round-6 evidence (developer tool, GPU box): default bench, optionally the 250k-pixel tile parity
# run (PARITY=1).  Each GPU step has its own time limit; the first failure ends the session.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
T=${TAG:-r06ev}
timeout -k 10 500 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
python3 tools/bench_brief.py gpurun_out/${T}_bench.json
tail -3 gpurun_out/${T}_bench.err
if [ "${PARITY:-0}" = 1 ]; then
timeout -k 10 900 python -u tools/tile_parity.py --batch 6 --out gpurun_out/${T}_tile_parity.json > gpurun_out/${T}_tile_parity.log 2>&1 || { echo "parity rc=$?"; tail -20 gpurun_out/${T}_tile_parity.log; exit 1; }
tail -1 gpurun_out/${T}_tile_parity.log
fi
