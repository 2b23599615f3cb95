#!/bin/bash
# Diagnostic GPU session: diag-build parity probe + per-phase cycle split (C3, C5), then PMC passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG=${1:-diag}
CCDGPU_LIBRARY="$R/lcmap-firebird_amd/lib/libccdgpu_diag.so" timeout -k 10 300 python tools/gpu_quick.py 256 > "$OUT/${TAG}_diagparity.log" 2>&1 &&
timeout -k 10 300 python tools/phase_profile.py 3 2 > "$OUT/${TAG}_phase_c3.json" 2>&1 &&
timeout -k 10 300 python tools/phase_profile.py 5 2 > "$OUT/${TAG}_phase_c5.json" 2>&1 &&
bash tools/gpu_pmc.sh "${TAG}_pmc"
rc=$?; echo "rc=$rc" > "$OUT/${TAG}_rc.txt"; exit $rc
