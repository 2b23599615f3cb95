#!/bin/bash
# Round-6 tile-leg knob A/B (developer tool, GPU box): the tile leg alone, interleaved rounds of
# the values in VALS for the bench flag FLAG.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
T=${TAG:-tileab}
for r in 1 2; do
  for v in $VALS; do
    timeout -k 10 300 python -u bench.py --no-resident --no-tile-lossless --tile-parity-pixels 0 $FLAG $v > gpurun_out/${T}_${v}_$r.json 2> gpurun_out/${T}_${v}_$r.err || { echo "tile $v rc=$?"; tail -20 gpurun_out/${T}_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/${T}_${v}_$r.json')); t=d['tile']; print('$FLAG $v round $r', round(t['value']), round(t['seconds'],2))"
  done
done
