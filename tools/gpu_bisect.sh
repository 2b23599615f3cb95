#!/bin/bash
# Round-2: w3/w4 golden check of each round-1 commit's library (lib/bisect/libr1_<sha>.so).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
for L in lcmap-firebird_amd/lib/bisect/libr1_*.so; do
  b=$(basename $L .so)
  timeout -k 10 120 python -u tools/r1_variant_repro.py $PWD/$L w3,w4 > gpurun_out/bisect_$b.json 2> gpurun_out/bisect_$b.err || { echo "rc=$? $b"; tail -5 gpurun_out/bisect_$b.err; exit 1; }
  python -c "
import json; r=json.load(open('gpurun_out/bisect_$b.json'))
print('$b', 'w4 problems', sum(x['golden_problems'] for x in r['w4'].values()), 'identical', all(x['identical_to_w3'] for x in r['w4'].values()))"
done
