#!/bin/bash
# Developer tool (GPU box): tile-leg A/B of environment settings, rounds interleaved.  Each
# argument is "tag:VAR=value,VAR2=value" ("tag:" alone = the defaults); every run is
# `bench.py --no-resident --no-tile-lossless` under its own time limit.  Usage:
#   TAG=r04b ROUNDS=2 tools/gpu_ab_tile.sh inplace: decode:CCDGPU_DECODE=1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=gpurun_out/${TAG:-abt}; mkdir -p $O
for r in $(seq 1 ${ROUNDS:-2}); do
  for spec in "$@"; do
    tag=${spec%%:*}; envs=${spec#*:}
    env $(echo "$envs" | tr ',' ' ') timeout -k 10 300 python -u bench.py --no-resident --no-tile-lossless --steps ${STEPS:-5} --warmup 1 ${BENCH_ARGS} > $O/${tag}_$r.json 2> $O/${tag}_$r.err || { echo "rc=$? $tag"; tail -5 $O/${tag}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${tag}_$r.json')); t=d['tile']; print('$tag', $r, round(d['value']), 's', round(t['seconds'],2), 'parity', t.get('parity_sample', {}) and {k: t['parity_sample'][k] for k in ('pixels','int_mismatches','float_mismatches','max_rel')}, t['worker_seconds_rank0'])"
  done
done
