#!/bin/bash
# Round-6 kernel A/B (developer tool, GPU box): GPU suite on the in-tree library, byte comparison
# against the baseline library (tools/lib_diff.py), resident A/B on C5 and C3 (tools/gpu_ab.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
T=${TAG:-kab}
BASE=${BASE:-lib/r6base/libccdgpu_base.so}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
timeout -k 10 300 python -u tools/lib_diff.py $BASE lib/libccdgpu.so > gpurun_out/${T}_diff.txt 2>&1; rc=$?
tail -8 gpurun_out/${T}_diff.txt
[ $rc -le 1 ] || { echo "lib_diff rc=$rc"; exit 1; }
NO_TESTS=1 TAG=$T LIBS="$BASE lib/libccdgpu.so" bash tools/gpu_ab.sh
