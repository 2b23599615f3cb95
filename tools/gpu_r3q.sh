#!/bin/bash
# Round-3 GPU call Q: tile-leg knobs with the unread encoding (contexts x encode threads x
# upload depth), then the default bench command (with its tile_lossless run).
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r03q; mkdir -p $O
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 240 python -u bench.py --no-resident --steps 5 --warmup 1 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "rc=$? $tag"; tail -3 $O/$tag.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); t=d['tile']; e=t.get('transport_encoding') or {}; print('$tag', round(d['value']), 's', round(t['seconds'],2), t['worker_seconds_rank0'], e.get('encode_thread_seconds_rank0'))"
}
run c3t4 --tile-contexts 3 --tile-copy-threads 4 || exit 1
run c4t3 --tile-contexts 4 --tile-copy-threads 3 || exit 1
run c4t4 --tile-contexts 4 --tile-copy-threads 4 || exit 1
run c5t3 --tile-contexts 5 --tile-copy-threads 3 || exit 1
run c3t4d3 --tile-contexts 3 --tile-copy-threads 4 --tile-depth 3 || exit 1
run c4t3b12 --tile-contexts 4 --tile-copy-threads 3 --tile-batch 12 || exit 1
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', round(d['value']), round(d['value_resident']), d['roofline']['frac'], d['tile']['seconds'], d.get('tile_lossless', {}).get('value'))"
echo done
