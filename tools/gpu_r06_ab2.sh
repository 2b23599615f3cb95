#!/bin/bash
# Round-6 kernel A/B, part 2 (developer tool, GPU box): byte comparison of each library in LIBS
# against the baseline (tools/lib_diff.py), then resident A/B rounds on C3 and C5
# (tools/ab_resident.py); no GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
T=${TAG:-ab2}
BASE=${BASE:-lib/r6base/libccdgpu_base.so}
for L in $LIBS; do
  [ "$L" = "$BASE" ] && continue
  timeout -k 10 300 python -u tools/lib_diff.py $BASE $L --chips ${DIFF_CHIPS:-3:0,3:3,5:1,5:4,2:0,4:1} > gpurun_out/${T}_diff_$(basename $L .so).txt 2>&1; rc=$?
  echo "== $L"; tail -4 gpurun_out/${T}_diff_$(basename $L .so).txt
  [ $rc -le 1 ] || { echo "lib_diff rc=$rc"; exit 1; }
done
timeout -k 10 400 python -u tools/ab_resident.py --config 3 --chips 64 --steps 6 --rounds ${ROUNDS:-2} $LIBS > gpurun_out/${T}_ab_c3.txt 2>&1 || { echo "ab c3 rc=$?"; tail -20 gpurun_out/${T}_ab_c3.txt; exit 1; }
grep round gpurun_out/${T}_ab_c3.txt
timeout -k 10 400 python -u tools/ab_resident.py --config 5 --chips 32 --steps 3 --rounds ${ROUNDS:-2} $LIBS > gpurun_out/${T}_ab_c5.txt 2>&1 || { echo "ab c5 rc=$?"; tail -20 gpurun_out/${T}_ab_c5.txt; exit 1; }
grep round gpurun_out/${T}_ab_c5.txt
