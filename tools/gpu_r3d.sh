#!/bin/bash
# Round-3 GPU call D: suite, full-tile parity (2500 distinct generated chips, 100 px per chip vs
# the C oracle), the driver's bench command, out-of-line CD A/B.
set -o pipefail
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest rc=$?" | tee $O/pytest_rc.txt
timeout -k 10 700 python -u tools/tile_parity.py --chips 2500 --sample 100 --out $O/tile_parity.json > $O/tile_parity.log 2>&1
echo "tile parity rc=$?" | tee -a $O/pytest_rc.txt
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -5 $O/bench.err; exit 1; }
L="lib/libccdgpu.so lib/libccdgpu.so:w4 lib/exp/libccdgpu_cdcall.so"
timeout -k 10 300 python -u tools/ab_resident.py --config 3 --chips 64 --steps 8 --rounds 1 $L > $O/ab_c3.txt 2> $O/ab_c3.err || { echo "ab c3 rc=$?"; exit 1; }
timeout -k 10 300 python -u tools/ab_resident.py --config 5 --chips 32 --steps 4 --rounds 1 $L > $O/ab_c5.txt 2> $O/ab_c5.err || { echo "ab c5 rc=$?"; exit 1; }
echo done
