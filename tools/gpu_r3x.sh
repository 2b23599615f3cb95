#!/bin/bash
# Round-3 GPU call X: rows fetched into reusable pinned buffers; workers stage uploads while their
# detection runs (ccdgpu_run_slot_begin /
# _query / _end): GPU suite, tile runs (4x3 default twice, 4x4, 6x2), kernel + copy timeline.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r03x; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 240 python -u bench.py --no-resident --no-tile-lossless --steps 5 --warmup 1 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "rc=$? $tag"; tail -3 $O/$tag.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); t=d['tile']; print('$tag', round(d['value']), 's', round(t['seconds'],2), t['worker_seconds_rank0'], t.get('cgroup_cpu_during_tile_s', {}).get('usage_s'))"
}
run c4t3 && run c4t4 --tile-copy-threads 4 && run c6t2 --tile-contexts 6 --tile-copy-threads 2 && run c4t3b || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace -o run -- python3 $R/bench.py --no-resident --no-tile-lossless --steps 5 --warmup 1 > $O/tile_traced.json 2> $O/tile_traced.err || { echo "trace rc=$?"; tail -5 $O/tile_traced.err; exit 1; }
cd $R
python3 tools/tile_timeline.py $O/trace/run_results.db $O/tile_traced.json > $O/timeline.json && cat $O/timeline.json
echo done
