#!/bin/bash
# Round-5 tile timeline at HEAD (developer tool, GPU box): one traced tile run (rocprofv3 kernel +
# memory-copy trace, no counters) and its timeline summary (tools/tile_timeline.py): the share of
# the timed window with a detection in flight, with an upload in flight, both, neither; H2D rate.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
O=gpurun_out/${TAG:-r05tl}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d $R/$O/trace -o run -- python3 $R/bench.py --no-resident --no-tile-lossless --no-cpu-baseline --steps 5 --warmup 1 > $R/$O/tile_traced.json 2> $R/$O/tile_traced.err || { echo "trace rc=$?"; tail -5 $R/$O/tile_traced.err; exit 1; }
cd $R
python3 tools/tile_timeline.py $O/trace/run_results.db $O/tile_traced.json > $O/tile_timeline.json || { echo "timeline failed"; exit 1; }
cat $O/tile_timeline.json
rm -rf $O/trace
