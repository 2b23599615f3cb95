#!/bin/bash
# Round-3 GPU call B: suite (narrowed EXEC assertions, device generator, paired Tmask), round-1
# EXEC probe, resident C3/C5 rates, full bench.
set -o pipefail
O=gpurun_out/r03b
mkdir -p $O
E=lcmap-firebird_amd/lib/exp
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest rc=$?" | tee $O/pytest_rc.txt
for v in w3 w4; do
  timeout -k 10 120 python -u tools/r1_exec_check.py $PWD/$E/libr1_475_xl.so $v >> $O/r1_exec.txt 2>&1 || { echo "rc=$? r1 $v" >> $O/r1_exec.txt; exit 1; }
done
for c in 3 5; do
  timeout -k 10 300 python -u bench.py --no-tile --no-packer --no-cpu-baseline --config $c --steps 10 --warmup 2 > $O/res_c$c.json 2> $O/res_c$c.err || { echo "resident c$c failed"; exit 1; }
done
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo bench failed; exit 1; }
echo done
