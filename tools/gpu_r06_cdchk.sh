#!/bin/bash
# Round-6 coordinate-descent stopping-test statistics (developer tool, GPU box): the
# CCD_CD_CHKSTAT diagnostic build on C3 and C5 chips (tools/phase_profile.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
L=$PWD/lcmap-firebird_amd/lib/diag6/libccdgpu_cdchk.so
CCDGPU_LIBRARY=$L CCD_DIAG_LIB=libccdgpu_cdchk.so timeout -k 10 300 python -u tools/phase_profile.py 3 4 > gpurun_out/cdchk_c3.json || exit 1
CCDGPU_LIBRARY=$L CCD_DIAG_LIB=libccdgpu_cdchk.so timeout -k 10 300 python -u tools/phase_profile.py 5 2 > gpurun_out/cdchk_c5.json || exit 1
grep -h "cd \|lasso cd\|spec early\|detect_ms" gpurun_out/cdchk_c3.json gpurun_out/cdchk_c5.json
