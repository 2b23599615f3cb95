#!/bin/bash
# Round-3 GPU call T: decode kernel with register palette + unrolled chunks: encode tests, tile
# run with the kernel/copy timeline, then the plain tile leg.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r03t; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_tile.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace -o run -- python3 $R/bench.py --no-resident --steps 5 --warmup 1 > $O/tile_traced.json 2> $O/tile_traced.err || { echo "trace rc=$?"; tail -5 $O/tile_traced.err; exit 1; }
cd $R
python3 tools/tile_timeline.py $O/trace/run_results.db $O/tile_traced.json
timeout -k 10 240 python -u bench.py --no-resident --steps 5 --warmup 1 > $O/tile.json 2> $O/tile.err || { echo "tile rc=$?"; exit 1; }
python3 -c "import json; d=json.load(open('$O/tile.json')); print('tile', round(d['value']), d['tile']['seconds'])"
echo done
