#!/bin/bash
# Round-3 GPU call J: GPU suite at the one-fit-site kernel, then resident A/B against the previous
# product library (lib/exp/libccdgpu_base.so) on C3 and C5, and the C5 phase split with the new
# counters (init / spec / refit counts).
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r03j; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L="lib/exp/libccdgpu_base.so lib/libccdgpu.so lib/exp/libccdgpu_nopair.so"
timeout -k 10 300 python -u tools/ab_resident.py --config 3 --chips 64 --steps 6 --rounds 2 $L > $O/ab_c3.txt 2> $O/ab_c3.err || { echo "ab c3 rc=$?"; tail -5 $O/ab_c3.err; exit 1; }
timeout -k 10 300 python -u tools/ab_resident.py --config 5 --chips 64 --steps 3 --rounds 2 $L > $O/ab_c5.txt 2> $O/ab_c5.err || { echo "ab c5 rc=$?"; tail -5 $O/ab_c5.err; exit 1; }
grep px/s $O/ab_c3.txt $O/ab_c5.txt
timeout -k 10 200 python -u tools/phase_profile.py 5 2 > $O/phase_c5.json 2> $O/phase_c5.err || { echo "phase c5 rc=$?"; exit 1; }
timeout -k 10 200 python -u tools/phase_profile.py 3 4 > $O/phase_c3.json 2> $O/phase_c3.err || { echo "phase c3 rc=$?"; exit 1; }
echo done
