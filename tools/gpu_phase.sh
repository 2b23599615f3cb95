#!/bin/bash
# Developer tool: diag-build golden parity, then the per-phase cycle split on C3 and C5 chips.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG=${1:-ph}
rm -f "$OUT/vc.log"
CCDGPU_LIBRARY="$R/lcmap-firebird_amd/lib/libccdgpu_diag.so" timeout -k 10 60 python tools/variant_check.py > "$OUT/${TAG}_diagparity.log" 2>&1 &&
timeout -k 10 200 python tools/phase_profile.py 3 2 > "$OUT/${TAG}_phase_c3.json" 2>&1 &&
timeout -k 10 200 python tools/phase_profile.py 5 2 > "$OUT/${TAG}_phase_c5.json" 2>&1
