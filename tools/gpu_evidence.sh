#!/bin/bash
# GPU evidence at HEAD (one gpurun call): GPU suite, smoke, the driver's default bench, a
# single-context rocprofv3 kernel-stats pass of the resident leg (its average dispatch duration is
# the per-launch duration behind bench.py's roofline), and -- with PMC=1 -- the PMC passes of
# tools/gpu_pmc.sh over the bench's resident workload key (summarised here by
# tools/pmc_summary.py --write into profiles/pmc_detect.json).  Usage: tools/gpu_evidence.sh TAG
set -o pipefail
TAG=${1:-ev}
R=$(pwd); O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
grep -o "full-size tile parity.*" $O/pytest.log | head -2
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('bench', round(d['value']), 'resident', round(d['value_resident']), 'frac', round(r['frac'],4), 'launch_ms', round(r['kernel_ms_per_launch'],2), 'tile_s', round(d['tile']['seconds'],2), 'parity', d['tile'].get('parity_sample'), 'lossless', d.get('tile_lossless', {}).get('value'))"
PMC=${PMC:-0} bash tools/gpu_evidence_stats.sh $TAG || exit 1
echo done
