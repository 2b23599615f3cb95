#!/bin/bash
# Round-3 GPU call M: parity of the initialize-fit-at-the-catch-site kernel (golden, chip and
# parameter tests through lib/exp/libccdgpu_initm.so), resident A/B: HEAD vs initm vs the same two
# without the 6-coefficient sweep specialisation.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r03m; mkdir -p $O
CCDGPU_LIBRARY=$R/lcmap-firebird_amd/lib/exp/libccdgpu_initm_nopc5.so timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q -k "not native_library" --timeout 120 --timeout-method thread > $O/pytest_initm_nopc5.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_initm_nopc5.log; exit 1; }
tail -1 $O/pytest_initm_nopc5.log
L="lib/libccdgpu.so lib/exp/libccdgpu_initm.so lib/exp/libccdgpu_initm_nopc5.so lib/exp/libccdgpu_head_nopc5.so"
timeout -k 10 300 python -u tools/ab_resident.py --config 3 --chips 64 --steps 6 --rounds 2 $L > $O/ab_c3.txt 2> $O/ab_c3.err || { echo "ab c3 rc=$?"; tail -5 $O/ab_c3.err; exit 1; }
timeout -k 10 300 python -u tools/ab_resident.py --config 5 --chips 64 --steps 3 --rounds 2 $L > $O/ab_c5.txt 2> $O/ab_c5.err || { echo "ab c5 rc=$?"; tail -5 $O/ab_c5.err; exit 1; }
grep px/s $O/ab_c3.txt $O/ab_c5.txt
echo done
