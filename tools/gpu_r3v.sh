#!/bin/bash
# Round-3 GPU call V: CU-reserved streams (upload decode + every launch kernel but detection) as
# the runner default (copy_cus 8): GPU suite,
# smoke, the driver's default bench, tile runs at 8 / 0 / 16 reserved CUs, and the kernel + copy
# timeline of a tile run with the default.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r03v; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', round(d['value']), 'lossless', d.get('tile_lossless', {}).get('value'), 'resident', d.get('value_resident'), d['roofline']['frac'])"
run() {  # tag, reserved CUs
  timeout -k 10 240 python -u bench.py --no-resident --no-tile-lossless --steps 5 --warmup 1 --tile-copy-cus $2 > $O/$1.json 2> $O/$1.err || { echo "rc=$? $1"; tail -3 $O/$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); t=d['tile']; print('$1', round(d['value']), 's', round(t['seconds'],2), t['worker_seconds_rank0'])"
}
run c8 8 && run c0 0 && run c16 16 && run c8b 8 && run c0b 0 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace -o run -- python3 $R/bench.py --no-resident --no-tile-lossless --steps 5 --warmup 1 > $O/tile_traced.json 2> $O/tile_traced.err || { echo "trace rc=$?"; tail -5 $O/tile_traced.err; exit 1; }
cd $R
python3 tools/tile_timeline.py $O/trace/run_results.db $O/tile_traced.json > $O/timeline.json && cat $O/timeline.json
echo done
