#!/bin/bash
# Round-2: full GPU tests on the gap-buffer kernel, the round-1 w4 reproduction, A/B bench vs the
# pre-gap kernel, full bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_d.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_d.log; exit 1; }
tail -3 gpurun_out/pytest_d.log
for L in libr1_475_fast.so libr1_475_on.so; do
  timeout -k 10 300 python -u tools/r1_variant_repro.py $L > gpurun_out/repro_$L.json 2> gpurun_out/repro_$L.err || { echo "repro rc=$? $L"; tail -20 gpurun_out/repro_$L.err; exit 1; }
done
CCDGPU_LIBRARY=$PWD/lcmap-firebird_amd/lib/libccdgpu_nogap.so timeout -k 10 600 python -u bench.py --steps 4 --no-cpu-baseline --no-tile --no-stream --no-packer > gpurun_out/bench_nogap.json 2> gpurun_out/bench_nogap.err || { echo "bench nogap rc=$?"; tail -20 gpurun_out/bench_nogap.err; exit 1; }
cat gpurun_out/bench_nogap.json
timeout -k 10 900 python -u bench.py --steps 4 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
