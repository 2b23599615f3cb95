#!/bin/bash
# Round-3 GPU call K: suite at the snow-through-catch + interleaved-check kernel, resident A/B
# (pre-dedup base, one-fit-site, current), C5 phase split, PMC passes on C3 and C5 of the current
# kernel, tile-leg variants (3 contexts, fewer copy threads, CPU quota of 16 on the box; host threads on the GPU NUMA node or not).
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r03k; mkdir -p $O
L="lib/exp/libccdgpu_base.so lib/exp/libccdgpu_onefit.so lib/libccdgpu.so lib/libccdgpu.so:w4"
timeout -k 10 300 python -u tools/ab_resident.py --config 3 --chips 64 --steps 6 --rounds 2 $L > $O/ab_c3.txt 2> $O/ab_c3.err || { echo "ab c3 rc=$?"; tail -5 $O/ab_c3.err; exit 1; }
timeout -k 10 300 python -u tools/ab_resident.py --config 5 --chips 64 --steps 3 --rounds 2 $L > $O/ab_c5.txt 2> $O/ab_c5.err || { echo "ab c5 rc=$?"; tail -5 $O/ab_c5.err; exit 1; }
grep px/s $O/ab_c3.txt $O/ab_c5.txt
timeout -k 10 200 python -u tools/phase_profile.py 5 2 > $O/phase_c5.json 2> $O/phase_c5.err || { echo "phase c5 rc=$?"; exit 1; }
CCD_DIAG_LIB=libccdgpu_cdcyc.so timeout -k 10 200 python -u tools/phase_profile.py 3 4 > $O/cdcyc_c3.json 2> $O/cdcyc_c3.err || { echo "cdcyc c3 rc=$?"; exit 1; }
CCD_DIAG_LIB=libccdgpu_cdcyc.so timeout -k 10 200 python -u tools/phase_profile.py 5 2 > $O/cdcyc_c5.json 2> $O/cdcyc_c5.err || { echo "cdcyc c5 rc=$?"; exit 1; }
grep -h "max_iter\|mean" $O/cdcyc_c3.json $O/cdcyc_c5.json
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 240 python -u bench.py --no-resident --steps 5 --warmup 1 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "rc=$? $tag"; tail -3 $O/$tag.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); t=d['tile']; print('$tag', round(d['value']), 's', round(t['seconds'],2), t['worker_seconds_rank0'])"
}
run c3t4 --tile-contexts 3 --tile-copy-threads 4 || exit 1
run c3t4nonuma --tile-contexts 3 --tile-copy-threads 4 --tile-no-numa || exit 1
run c4t3 --tile-contexts 4 --tile-copy-threads 3 --tile-depth 1 || exit 1
TAG=r03k_c3 CONFIG=3 CHIPS=64 bash tools/gpu_pmc.sh r03k_c3 || { echo "pmc c3 failed"; exit 1; }
TAG=r03k_c5 CONFIG=5 CHIPS=64 bash tools/gpu_pmc.sh r03k_c5 || { echo "pmc c5 failed"; exit 1; }
echo done
