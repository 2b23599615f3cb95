#!/bin/bash
# Round-2: parity tests + A/B bench (pre-gap vs gap kernel) + phase split after a kernel change.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export CCD_BENCH_CACHE=/tmp/ccd_bench_cache
timeout -k 10 900 python -u -m pytest tests/test_gpu.py tests/test_gpu_batches.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_e.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_e.log; exit 1; }
tail -2 gpurun_out/pytest_e.log
Q="--steps 4 --no-cpu-baseline --no-tile --no-stream --no-packer"
for L in ${LIBS:-libccdgpu_nogap libccdgpu}; do
  CCDGPU_LIBRARY=$PWD/lcmap-firebird_amd/lib/$L.so timeout -k 10 600 python -u bench.py $Q > gpurun_out/bench_$L.json 2> gpurun_out/bench_$L.err || { echo "bench rc=$? $L"; tail -20 gpurun_out/bench_$L.err; exit 1; }
  python -c "import json; b=json.load(open('gpurun_out/bench_$L.json')); print('$L', round(b['value']), round(b['roofline']['frac'],4), round(b['roofline']['kernel_ms_per_launch'],1))"
done
timeout -k 10 300 python tools/phase_profile.py 3 2 > gpurun_out/phase_e_c3.json 2>&1 || { echo "phase rc=$?"; exit 1; }
grep -E "compaction|cycles_per_pixel|detect_ms" gpurun_out/phase_e_c3.json
