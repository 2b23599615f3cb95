#!/bin/bash
# Round-2 (session 2): GPU suite at the working tree, resident A/B of the kernel libraries in
# LIBS, then the tile leg at upload depths 1 and 2.  Each GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export CCD_BENCH_CACHE=/tmp/ccd_bench_cache
T=${TAG:-r2h}
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
Q="--steps 4 --no-cpu-baseline --no-tile --no-stream --no-packer"
for n in ${LIBS:-libccdgpu}; do
  CCDGPU_LIBRARY=$PWD/lcmap-firebird_amd/lib/$n.so timeout -k 10 300 python -u bench.py $Q > gpurun_out/${T}_$n.json 2> gpurun_out/${T}_$n.err || { echo "bench rc=$? $n"; tail -20 gpurun_out/${T}_$n.err; exit 1; }
  python -c "import json; b=json.load(open('gpurun_out/${T}_$n.json')); print('$n', round(b['value']), round(b['roofline']['frac'],4), round(b['roofline']['kernel_ms_per_launch'],1))"
done
for dp in ${DEPTHS:-1 2}; do
  timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-stream --no-packer --tile-depth $dp > gpurun_out/${T}_tile_d$dp.json 2> gpurun_out/${T}_tile_d$dp.err || { echo "tile rc=$? $dp"; tail -20 gpurun_out/${T}_tile_d$dp.err; exit 1; }
  python -c "import json; b=json.load(open('gpurun_out/${T}_tile_d$dp.json'))['tile']; print('depth $dp', round(b['value']), round(b['seconds'],2), b['worker_seconds_rank0'])"
done
