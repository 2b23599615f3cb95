#!/bin/bash
# Developer tool: golden parity of each listed kernel library variant (lcmap-firebird_amd/lib/<v>.so),
# with the register budget named by KERNELS (w1 w2 w3).
set -o pipefail
for v in "$@"; do
  for kv in ${KERNELS:-w3}; do
    echo -n "$kv " >> gpurun_out/vc.log
    CCDGPU_KERNEL=$kv CCDGPU_LIBRARY=$PWD/lcmap-firebird_amd/lib/$v.so timeout -k 10 60 python tools/variant_check.py >> gpurun_out/vc.log 2>&1 || { echo "rc=$? $v" >> gpurun_out/vc.log; exit 1; }
  done
done
