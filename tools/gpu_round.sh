#!/bin/bash
# One GPU session: pytest -m gpu, smoke, bench, rocprofv3 kernel trace.  Each GPU step has its
# own time limit; steps are chained so that a failure stops the session.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT="$R/gpurun_out"
mkdir -p "$OUT"
TAG=${1:-r01}
STEPS=${STEPS:-all}
run_tests() { timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/${TAG}_pytest_gpu.log" 2>&1; }
run_smoke() { timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${TAG}_smoke.log" 2>&1; }
run_bench() { timeout -k 10 600 python bench.py > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err"; }
run_prof() {
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OUT/${TAG}_prof" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-stream --no-packer --no-tile --contexts 1 \
      > "$OUT/${TAG}_prof.log" 2>&1 )
}
case "$STEPS" in
  all) run_tests && run_smoke && run_bench && run_prof ;;
  tests) run_tests ;;
  bench) run_bench ;;
  prof) run_prof ;;
  benchprof) run_bench && run_prof ;;
esac
rc=$?
echo "rc=$rc" > "$OUT/${TAG}_rc.txt"
exit $rc
