set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r05d}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 400 python -u tools/ab_resident.py --config 5 --chips 64 --steps 4 --rounds 2 ${LIBS:-lib/libccdgpu.so lib/ab5/libccdgpu_r2.so} > gpurun_out/${T}_ab_c5.txt 2>&1 || { echo "ab c5 rc=$?"; tail -20 gpurun_out/${T}_ab_c5.txt; exit 1; }
grep round gpurun_out/${T}_ab_c5.txt
timeout -k 10 400 python -u tools/ab_resident.py --config 3 --chips 64 --steps 8 --rounds 2 ${LIBS:-lib/libccdgpu.so lib/ab5/libccdgpu_r2.so} > gpurun_out/${T}_ab_c3.txt 2>&1 || { echo "ab c3 rc=$?"; tail -20 gpurun_out/${T}_ab_c3.txt; exit 1; }
grep round gpurun_out/${T}_ab_c3.txt
CCDGPU_LIBRARY=$PWD/lcmap-firebird_amd/lib/ab5/libccdgpu_diag.so timeout -k 10 300 python -u tools/phase_profile.py 5 2 > gpurun_out/${T}_phase_c5.json 2> gpurun_out/${T}_phase_c5.err || { echo "phase c5 rc=$?"; tail -5 gpurun_out/${T}_phase_c5.err; exit 1; }
CCDGPU_LIBRARY=$PWD/lcmap-firebird_amd/lib/ab5/libccdgpu_diag.so timeout -k 10 300 python -u tools/phase_profile.py 3 4 > gpurun_out/${T}_phase_c3.json 2> gpurun_out/${T}_phase_c3.err || { echo "phase c3 rc=$?"; tail -5 gpurun_out/${T}_phase_c3.err; exit 1; }
echo phases ok
