#!/bin/bash
# Round-6 host-side probes (developer tool, GPU box): the tile leg alone with the default libgomp
# wait policy and with OMP_WAIT_POLICY=passive (per-thread CPU seconds of each run), then the
# bench at N = 2 ranks sharing the one GPU (rehearsal of the driver's N > 1 path, with the
# other-config resident legs).  Each step has its own time limit; the first failure ends it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
T=${TAG:-r06host}
for pol in default passive; do
  if [ $pol = passive ]; then export OMP_WAIT_POLICY=passive; fi
  timeout -k 10 300 python -u bench.py --no-resident --no-tile-lossless > gpurun_out/${T}_tile_${pol}.json 2> gpurun_out/${T}_tile_${pol}.err || { echo "tile $pol rc=$?"; tail -20 gpurun_out/${T}_tile_${pol}.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${T}_tile_${pol}.json')); t=d['tile']; print('$pol', round(t['value']), round(t['seconds'],2), t['cgroup_cpu_during_tile_s']['usage_s'], t['thread_cpu_during_tile_rank0']['by_thread_s'])"
done
unset OMP_WAIT_POLICY
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --share-device --no-cpu-baseline > gpurun_out/${T}_n2.json 2> gpurun_out/${T}_n2.err || { echo "n2 rc=$?"; tail -30 gpurun_out/${T}_n2.err; exit 1; }
python3 tools/bench_brief.py gpurun_out/${T}_n2.json
