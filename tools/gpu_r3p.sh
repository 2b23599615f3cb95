#!/bin/bash
# Round-3 GPU call P: suite (incl. the unread-drop encoding test), tile leg with the 'unread'
# encoding (runner default) vs 'lossless', contexts 3/4, and the default bench command.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r03p; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 240 python -u bench.py --no-resident --steps 5 --warmup 1 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "rc=$? $tag"; tail -3 $O/$tag.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); t=d['tile']; e=t.get('transport_encoding') or {}; print('$tag', round(d['value']), 's', round(t['seconds'],2), t['worker_seconds_rank0'], e.get('sent_over_raw'), e.get('encode_thread_seconds_rank0'))"
}
run unread || exit 1
run lossless --tile-encode lossless || exit 1
run unread_c4 --tile-contexts 4 --tile-copy-threads 3 || exit 1
run unread_b16 --tile-batch 16 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', round(d['value']), round(d['value_resident']), d['roofline']['frac'], d['tile']['seconds'])"
echo done
