#!/bin/bash
# Round-3 GPU call S: timeline of the tile leg (kernel + memory-copy trace, no counters): how much
# of the tile's wall time the detection kernels and the H2D copies cover.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r03s; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace -o run -- python3 $R/bench.py --no-resident --steps 5 --warmup 1 > $O/tile.json 2> $O/tile.err || { echo "trace rc=$?"; tail -5 $O/tile.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/tile.json')); print('tile', round(d['value']), d['tile']['seconds'])"
echo done
