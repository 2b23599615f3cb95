#!/bin/bash
# Round-3 GPU call I: host topology of the box (GPU NUMA node, node CPU lists, our affinity),
# then tile-leg knob sweep at HEAD (streamed pool copies): copy threads, contexts, batch size.
set -o pipefail
O=gpurun_out/r03i
mkdir -p $O
{
  echo "affinity: $(python3 -c 'import os; s=sorted(os.sched_getaffinity(0)); print(len(s), s[:4], s[-4:])')"
  for f in /sys/class/drm/card*/device/numa_node; do echo "$f $(cat $f 2>/dev/null)"; done
  for n in /sys/devices/system/node/node*/cpulist; do echo "$n $(cat $n)"; done
  cat /sys/fs/cgroup/cpu.max 2>/dev/null
  grep -E "MemTotal|MemAvailable" /proc/meminfo
} > $O/topo.txt 2>&1
cat $O/topo.txt
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 240 python -u bench.py --no-resident --steps 5 --warmup 1 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "rc=$? $tag"; tail -3 $O/$tag.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); t=d['tile']; print('$tag', round(d['value']), 's', round(t['seconds'],2), t['worker_seconds_rank0'])"
}
run base || exit 1
run copy16 --tile-copy-threads 16 || exit 1
run ctx3 --tile-contexts 3 || exit 1
run ctx3copy4 --tile-contexts 3 --tile-copy-threads 4 || exit 1
run b16 --tile-batch 16 || exit 1
echo done
