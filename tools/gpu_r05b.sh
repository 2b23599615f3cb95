set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05b_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/r05b_pytest.log; exit 1; }
tail -3 gpurun_out/r05b_pytest.log
timeout -k 10 400 python -u tools/ab_resident.py --config 3 --chips 64 --steps 8 --rounds 2 lib/libccdgpu.so lib/ab5/libccdgpu_r2.so lib/ab5/libccdgpu_rs6.so lib/ab5/libccdgpu_rs8.so > gpurun_out/r05b_ab_c3.txt 2>&1 || { echo "ab c3 rc=$?"; tail -20 gpurun_out/r05b_ab_c3.txt; exit 1; }
grep round gpurun_out/r05b_ab_c3.txt
timeout -k 10 400 python -u tools/ab_resident.py --config 5 --chips 64 --steps 4 --rounds 2 lib/libccdgpu.so lib/ab5/libccdgpu_r2.so > gpurun_out/r05b_ab_c5.txt 2>&1 || { echo "ab c5 rc=$?"; tail -20 gpurun_out/r05b_ab_c5.txt; exit 1; }
grep round gpurun_out/r05b_ab_c5.txt
timeout -k 10 400 python -u bench.py > gpurun_out/r05b_bench.json 2> gpurun_out/r05b_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/r05b_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r05b_bench.json')); print('tile', d['value'], 'resident', d['value_resident'], 'frac', d['roofline']['frac'], d['tile']['parity_sample'])"
