#!/bin/bash
# Round-6 A/B (developer tool, GPU box): the encoder's streaming (non-temporal) stores of the band
# runs vs ordinary stores (CCDGPU_ENCODE_NT=0): encode tests on the AVX-512 path, encoder
# throughput, then the tile leg alone with each.  Each step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
T=${TAG:-r06nt}
timeout -k 10 300 python -u -m pytest tests/test_encode.py tests/test_gpu_encode.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
for nt in 0 1; do
  CCDGPU_ENCODE_NT=$nt timeout -k 10 300 python -u tools/encode_bench.py 6 3 > gpurun_out/${T}_enc_nt$nt.txt 2>&1 || { echo "enc rc=$?"; tail gpurun_out/${T}_enc_nt$nt.txt; exit 1; }
  echo "nt=$nt $(tail -1 gpurun_out/${T}_enc_nt$nt.txt)"
done
for nt in 0 1 0 1; do
  CCDGPU_ENCODE_NT=$nt timeout -k 10 300 python -u bench.py --no-resident --no-tile-lossless > gpurun_out/${T}_tile_nt$nt.json 2> gpurun_out/${T}_tile_nt$nt.err || { echo "tile rc=$?"; tail -20 gpurun_out/${T}_tile_nt$nt.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${T}_tile_nt$nt.json')); t=d['tile']; print('nt=$nt', round(t['value']), round(t['seconds'],2), t['cgroup_cpu_during_tile_s']['usage_s'], t['transport_encoding']['encode_thread_seconds_rank0'], t['thread_cpu_during_tile_rank0']['by_thread_s'])"
done
