#!/bin/bash
# Round-2: register-budget variants of the current kernel on the bench workload.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export CCD_BENCH_CACHE=/tmp/ccd_bench_cache
Q="--steps 4 --no-cpu-baseline --no-tile --no-stream --no-packer"
for K in ${KS:-w3 w4 w2}; do
  CCDGPU_KERNEL=$K timeout -k 10 600 python -u bench.py $Q > gpurun_out/knob_$K.json 2> gpurun_out/knob_$K.err || { echo "bench rc=$? $K"; tail -20 gpurun_out/knob_$K.err; exit 1; }
  python -c "import json; b=json.load(open('gpurun_out/knob_$K.json')); print('$K', round(b['value']), round(b['roofline']['frac'],4), round(b['roofline']['kernel_ms_per_launch'],1))"
done
