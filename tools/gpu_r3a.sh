#!/bin/bash
# Round-3 GPU call A: suite at HEAD (EXEC-restore fix + EXEC assertions in the guard build),
# the w4 reproducer with and without the fix, round-1's 475ecd7 w4 with and without, smoke, bench.
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r03a
mkdir -p $O
E=lcmap-firebird_amd/lib/exp
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest rc=$?" | tee $O/pytest_rc.txt
for lib in libccdgpu_repro.so libccdgpu_reprofix.so; do
  for v in w1 w2 w3 w4; do
    CCDGPU_LIBRARY=$PWD/$E/$lib CCDGPU_KERNEL=$v timeout -k 10 120 python -u tools/variant_check.py >> $O/repro.txt 2>&1 || { echo "rc=$? $lib $v" >> $O/repro.txt; exit 1; }
    echo " ^ $v" >> $O/repro.txt
  done
done
for lib in libr1_475_k.so libr1_475_kfix.so; do
  timeout -k 10 180 python -u tools/r1_variant_repro.py $PWD/$E/$lib w3,w4 > $O/r1_$lib.json 2> $O/r1_$lib.err || { echo "rc=$? r1 $lib"; exit 1; }
done
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo bench failed; exit 1; }
echo done
