#!/bin/bash
# Round-2: tile-leg knobs, full 2500-chip tile each.  Args: BATCHxCONTEXTS ... (default 8x2 8x3)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export CCD_BENCH_CACHE=/tmp/ccd_bench_cache
[ $# -eq 0 ] && set -- 8x2 8x3
for cfg in "$@"; do
  b=${cfg%x*}; c=${cfg#*x}
  timeout -k 10 600 python -u bench.py --steps 1 --warmup 0 --chips 16 --contexts 1 --no-cpu-baseline --no-stream --no-packer --tile-batch $b --tile-contexts $c > gpurun_out/tk_$cfg.json 2> gpurun_out/tk_$cfg.err || { echo "rc=$? $cfg"; tail -20 gpurun_out/tk_$cfg.err; exit 1; }
  python -c "import json; b=json.load(open('gpurun_out/tk_$cfg.json')); t=b['tile']; print('$cfg', round(t['value']), round(t['seconds'],2), t['worker_seconds_rank0'])"
done
