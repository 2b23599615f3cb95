#!/bin/bash
# Round-3 GPU call O: suite with blocking detection waits + vectorised encoder pass 1, then the tile
# leg encoded vs raw, then the default bench command.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r03o; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 240 python -u bench.py --no-resident --steps 5 --warmup 1 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "rc=$? $tag"; tail -3 $O/$tag.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); t=d['tile']; print('$tag', round(d['value']), 's', round(t['seconds'],2), t['worker_seconds_rank0'], t.get('transport_encoding'))"
}
run enc || exit 1
run raw --tile-no-encode || exit 1
run enc_t5 --tile-copy-threads 5 || exit 1
run enc2 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', round(d['value']), round(d['value_resident']), d['roofline']['frac'])"
echo done
