#!/bin/bash
# Round-3 GPU call Y (evidence at HEAD, in order of importance): GPU suite, smoke, the driver's
# default bench, rocprofv3 kernel stats of the resident leg, tile parity over 2500 distinct chips
# through the runner's defaults, tile knob runs, kernel + copy timeline of the tile leg.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r03y; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', round(d['value']), round(d['value_resident']), d['roofline']['frac'], d['tile']['seconds'], d.get('tile_lossless', {}).get('value'), d['tile']['worker_seconds_rank0'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats -o run -- python3 $R/bench.py --no-tile --no-packer --no-cpu-baseline --steps 10 --warmup 2 > $O/stats_bench.json 2> $O/stats_bench.err || { echo "stats rc=$?"; exit 1; }
cd $R
python3 tools/rocpd_stats.py $O/stats/run_results.db $O/kernel_stats.csv && head -4 $O/kernel_stats.csv
timeout -k 10 600 python -u tools/tile_parity.py --chips 2500 --sample 100 --out $O/tile_parity.json > $O/tile_parity.log 2>&1 || { echo "tile parity rc=$?"; tail -5 $O/tile_parity.log; exit 1; }
tail -1 $O/tile_parity.log | cut -c1-400
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 240 python -u bench.py --no-resident --no-tile-lossless --steps 5 --warmup 1 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "rc=$? $tag"; tail -3 $O/$tag.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); t=d['tile']; print('$tag', round(d['value']), 's', round(t['seconds'],2), t['worker_seconds_rank0'])"
}
run c4t3 && run c6t2 --tile-contexts 6 --tile-copy-threads 2 && run c4t4 --tile-copy-threads 4 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace -o run -- python3 $R/bench.py --no-resident --no-tile-lossless --steps 5 --warmup 1 > $O/tile_traced.json 2> $O/tile_traced.err || { echo "trace rc=$?"; tail -5 $O/tile_traced.err; exit 1; }
cd $R
python3 tools/tile_timeline.py $O/trace/run_results.db $O/tile_traced.json > $O/timeline.json && cat $O/timeline.json
echo done
