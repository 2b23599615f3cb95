#!/bin/bash
# Round-3 GPU call Y2 (short evidence at HEAD): GPU suite, smoke, the driver's
# default bench, rocprofv3 kernel stats of the resident leg, tile parity over 2500 distinct chips
# through the runner's defaults, tile knob runs, kernel + copy timeline of the tile leg.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r03y2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', round(d['value']), round(d['value_resident']), d['roofline']['frac'], d['tile']['seconds'], d.get('tile_lossless', {}).get('value'), d['tile']['worker_seconds_rank0'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats -o run -- python3 $R/bench.py --no-tile --no-packer --no-cpu-baseline --steps 10 --warmup 2 > $O/stats_bench.json 2> $O/stats_bench.err || { echo "stats rc=$?"; exit 1; }
echo done
