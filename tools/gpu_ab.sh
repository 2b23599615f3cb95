#!/bin/bash
# Developer tool: GPU suite at the working tree, then resident A/B of the kernel libraries in LIBS
# (lib/<name>.so) on the C3 tile mix and, with C5=1, on the change-dense C5 chips.  Each GPU step
# has its own time limit; the first failure ends the session.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
T=${TAG:-ab}
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
Q="--steps ${STEPS:-4} --no-cpu-baseline --no-tile --no-packer"
for cfg in 3 ${C5:+5}; do
  for n in ${LIBS:-libccdgpu}; do
    CCDGPU_LIBRARY=$PWD/lcmap-firebird_amd/lib/$n.so timeout -k 10 300 python -u bench.py $Q --config $cfg > gpurun_out/${T}_c${cfg}_$n.json 2> gpurun_out/${T}_c${cfg}_$n.err || { echo "bench rc=$? $n"; tail -20 gpurun_out/${T}_c${cfg}_$n.err; exit 1; }
    python -c "import json; b=json.load(open('gpurun_out/${T}_c${cfg}_$n.json')); print('C$cfg', '$n', round(b['value']), round(b['roofline']['frac'],4), round(b['roofline']['kernel_ms_per_launch'],1))"
  done
done
