#!/bin/bash
# Round-3 GPU call W: host encoder profile on the box's CPU (per pass, 1/3/6 threads, pass-2
# block 32 vs 1); tile knob sweep with CU-reserved contexts: contexts x encode threads, upload
# depth, launch size.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r03w; mkdir -p $O
timeout -k 10 120 python3 tools/encode_prof.py $O/encprof > $O/encode_prof.txt 2>&1 || { echo "encode_prof rc=$?"; tail -5 $O/encode_prof.txt; exit 1; }
cat $O/encode_prof.txt
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 240 python -u bench.py --no-resident --no-tile-lossless --steps 5 --warmup 1 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "rc=$? $tag"; tail -3 $O/$tag.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); t=d['tile']; print('$tag', round(d['value']), 's', round(t['seconds'],2), t['worker_seconds_rank0'], t.get('cgroup_cpu_during_tile_s', {}).get('usage_s'))"
}
run c4t3 && run c5t3 --tile-contexts 5 && run c6t2 --tile-contexts 6 --tile-copy-threads 2 && run c5t2 --tile-contexts 5 --tile-copy-threads 2 \
  && run c4t3d3 --tile-depth 3 && run c4t3b16 --tile-batch 16 && run c4t4 --tile-copy-threads 4 && run c4t3b || exit 1
echo done
