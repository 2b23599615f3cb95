#!/bin/bash
# Round-3 GPU call G (evidence at HEAD): GPU suite, smoke, the driver's default bench command,
# rocprofv3 kernel-trace stats of the resident leg.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r03g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats -o run -- python3 $R/bench.py --no-tile --no-packer --no-cpu-baseline --steps 10 --warmup 2 > $O/stats_bench.json 2> $O/stats_bench.err || { echo "stats rc=$?"; exit 1; }
echo done
