#!/bin/bash
# Round-3 GPU call U: suite with pinned per-launch copies; tile leg with CU-reserved copy streams
# (CCDGPU_COPY_CUS 0 / 8 / 16 / 32), cgroup CPU accounting per run.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r03u; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # tag, copy CUs, bench args...
  local tag=$1; local cus=$2; shift; shift
  CCDGPU_COPY_CUS=$cus timeout -k 10 240 python -u bench.py --no-resident --steps 5 --warmup 1 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "rc=$? $tag"; tail -3 $O/$tag.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); t=d['tile']; print('$tag', round(d['value']), 's', round(t['seconds'],2), t['worker_seconds_rank0'], t.get('cgroup_cpu_during_tile_s'))"
}
run cus0 0 || exit 1
run cus8 8 || exit 1
run cus16 16 || exit 1
run cus32 32 || exit 1
run cus0b 0 || exit 1
echo done
