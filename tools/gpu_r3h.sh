#!/bin/bash
# Round-3 GPU call H: resident A/B (product vs no-EXEC-fix vs no paired Tmask) on C3 and C5,
# per-phase split (diag build) of C3 and C5, PMC passes on C3 (bench key) and C5.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r03h; mkdir -p $O
L="lib/libccdgpu.so lib/exp/libccdgpu_nokfix.so lib/exp/libccdgpu_nopair.so"
timeout -k 10 300 python -u tools/ab_resident.py --config 3 --chips 64 --steps 6 --rounds 2 $L > $O/ab_c3.txt 2> $O/ab_c3.err || { echo "ab c3 rc=$?"; tail -5 $O/ab_c3.err; exit 1; }
timeout -k 10 300 python -u tools/ab_resident.py --config 5 --chips 64 --steps 3 --rounds 2 $L > $O/ab_c5.txt 2> $O/ab_c5.err || { echo "ab c5 rc=$?"; tail -5 $O/ab_c5.err; exit 1; }
grep px/s $O/ab_c3.txt $O/ab_c5.txt
timeout -k 10 200 python -u tools/phase_profile.py 3 4 > $O/phase_c3.json 2> $O/phase_c3.err || { echo "phase c3 rc=$?"; exit 1; }
timeout -k 10 200 python -u tools/phase_profile.py 5 2 > $O/phase_c5.json 2> $O/phase_c5.err || { echo "phase c5 rc=$?"; exit 1; }
TAG=r03h_c3 CONFIG=3 CHIPS=64 bash tools/gpu_pmc.sh r03h_c3 || { echo "pmc c3 failed"; exit 1; }
TAG=r03h_c5 CONFIG=5 CHIPS=64 bash tools/gpu_pmc.sh r03h_c5 || { echo "pmc c5 failed"; exit 1; }
echo done
