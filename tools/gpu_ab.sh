#!/bin/bash
# Developer tool (GPU box): GPU suite on the in-tree library, then resident A/B rounds of the
# libraries in LIBS on C5 and C3 (tools/ab_resident.py).  NO_TESTS=1 skips the suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
T=${TAG:-ab}
if [ -z "$NO_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
fi
timeout -k 10 400 python -u tools/ab_resident.py --config 5 --chips 64 --steps 3 --rounds 2 $LIBS > gpurun_out/${T}_ab_c5.txt 2>&1 || { echo "ab c5 rc=$?"; tail -20 gpurun_out/${T}_ab_c5.txt; exit 1; }
grep round gpurun_out/${T}_ab_c5.txt
timeout -k 10 400 python -u tools/ab_resident.py --config 3 --chips 64 --steps 6 --rounds 2 $LIBS > gpurun_out/${T}_ab_c3.txt 2>&1 || { echo "ab c3 rc=$?"; tail -20 gpurun_out/${T}_ab_c3.txt; exit 1; }
grep round gpurun_out/${T}_ab_c3.txt
