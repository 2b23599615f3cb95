set -o pipefail
for v in A B C; do
  L=$PWD/lcmap-firebird_amd/lib/exp/lib$v.so
  echo -n "$v " >> gpurun_out/exp_parity.log
  CCDGPU_LIBRARY=$L timeout -k 10 60 python tools/variant_check.py >> gpurun_out/exp_parity.log 2>&1 || exit 1
  CCDGPU_LIBRARY=$L timeout -k 10 200 python bench.py --steps 6 --no-cpu-baseline --no-packer --no-stream > gpurun_out/exp_$v.json 2>&1 || exit 1
done
