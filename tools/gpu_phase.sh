#!/bin/bash
# Developer tool: per-phase cycle split (diag build) on C3 and C5 chips.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG=${1:-ph}
timeout -k 10 200 python tools/phase_profile.py 3 2 > "$OUT/${TAG}_phase_c3.json" 2>&1 &&
timeout -k 10 200 python tools/phase_profile.py 5 2 > "$OUT/${TAG}_phase_c5.json" 2>&1
