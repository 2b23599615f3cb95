#!/bin/bash
# Round-3 GPU call C: resident A/B (fix / paired Tmask / round-2 kernel) on C3 and C5, the tile
# leg with the direct-write generator, phase profiles of C3 / C5.
set -o pipefail
O=gpurun_out/r03c
mkdir -p $O
E=lcmap-firebird_amd/lib/exp
L="lib/libccdgpu.so lib/exp/libccdgpu_nofix.so lib/exp/libccdgpu_nopair.so lib/exp/libccdgpu_r2.so"
timeout -k 10 400 python -u tools/ab_resident.py --config 3 --chips 64 --steps 8 --rounds 2 $L > $O/ab_c3.txt 2> $O/ab_c3.err || { echo "ab c3 rc=$?"; tail -5 $O/ab_c3.err; exit 1; }
timeout -k 10 400 python -u tools/ab_resident.py --config 5 --chips 32 --steps 4 --rounds 1 $L > $O/ab_c5.txt 2> $O/ab_c5.err || { echo "ab c5 rc=$?"; tail -5 $O/ab_c5.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-packer > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -5 $O/bench.err; exit 1; }
for c in 3 5; do
  timeout -k 10 200 python -u tools/phase_profile.py $c 2 > $O/phase_c$c.json 2> $O/phase_c$c.err || { echo "phase c$c rc=$?"; exit 1; }
done
echo done
