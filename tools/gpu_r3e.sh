#!/bin/bash
# Round-3 GPU call E: tile-leg knob sweep (contexts, batch, depth, SDMA vs blit copies), one
# process on one GPU, tile leg only.
set -o pipefail
O=gpurun_out/r03e
mkdir -p $O
run() {  # tag, env, args
  local tag=$1; shift
  env "$@" > /dev/null  # (validate env syntax)
  timeout -k 10 240 env "$@" python -u bench.py --no-resident --steps 10 --warmup 2 ${ARGS} > $O/$tag.json 2> $O/$tag.err || { echo "rc=$? $tag"; tail -3 $O/$tag.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); t=d['tile']; print('$tag', round(d['value']), 's', round(t['seconds'],2), t['worker_seconds_rank0'])"
}
ARGS="--tile-contexts 2 --tile-batch 8 --tile-depth 2" run c2b8d2 X=1 || exit 1
ARGS="--tile-contexts 3 --tile-batch 8 --tile-depth 2" run c3b8d2 X=1 || exit 1
ARGS="--tile-contexts 4 --tile-batch 8 --tile-depth 1" run c4b8d1 X=1 || exit 1
ARGS="--tile-contexts 2 --tile-batch 16 --tile-depth 2" run c2b16d2 X=1 || exit 1
ARGS="--tile-contexts 2 --tile-batch 8 --tile-depth 2" run c2b8d2_blit HSA_ENABLE_SDMA=0 || exit 1
ARGS="--tile-contexts 3 --tile-batch 8 --tile-depth 2" run c3b8d2_blit HSA_ENABLE_SDMA=0 || exit 1
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -5 $O/bench.err; exit 1; }
echo done
