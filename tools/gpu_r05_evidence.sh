#!/bin/bash
# Round-5 evidence at HEAD (developer tool, GPU box): GPU suite, smoke, default bench, the
# single-context rocprofv3 kernel-stats pass + PMC passes of the C3 resident workload, the C5 PMC
# passes (the C5 PMC passes and the tile parity run: tools/gpu_r05_parity.sh).  Each GPU step has its own time limit;
# the first failure ends the session.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
T=${TAG:-r05ev}
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
if [ -z "$NO_BENCH" ]; then
timeout -k 10 500 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); print('tile', round(d['value']), 'resident', round(d['value_resident']), 'frac', round(d['roofline']['frac'],4), 'ms', round(d['roofline']['kernel_ms_per_launch'],2), d['tile']['parity_sample']['int_mismatches'], d['tile']['parity_sample']['float_mismatches'])"
fi
PMC=1 bash tools/gpu_evidence_stats.sh ${T}_stats || { echo "stats/pmc failed"; exit 1; }
echo stats pmc ok
