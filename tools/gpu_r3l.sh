#!/bin/bash
# Round-3 GPU call L: suite at the spec-cut kernel (CCD_SPEC_CUT=8), resident A/B of the cut
# threshold (none / 4 / 8 / 16) on C5 and C3, C5 phase split.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r03l; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L="lib/exp/libccdgpu_nocut.so lib/exp/libccdgpu_cut4.so lib/libccdgpu.so lib/exp/libccdgpu_cut16.so"
timeout -k 10 300 python -u tools/ab_resident.py --config 5 --chips 64 --steps 3 --rounds 2 $L > $O/ab_c5.txt 2> $O/ab_c5.err || { echo "ab c5 rc=$?"; tail -5 $O/ab_c5.err; exit 1; }
timeout -k 10 300 python -u tools/ab_resident.py --config 3 --chips 64 --steps 6 --rounds 2 $L > $O/ab_c3.txt 2> $O/ab_c3.err || { echo "ab c3 rc=$?"; tail -5 $O/ab_c3.err; exit 1; }
grep px/s $O/ab_c3.txt $O/ab_c5.txt
timeout -k 10 200 python -u tools/phase_profile.py 5 2 > $O/phase_c5.json 2> $O/phase_c5.err || { echo "phase c5 rc=$?"; exit 1; }
echo done
