#!/bin/bash
# conv_tap16 (8 waves, 4 per SIMD) vs conv_tap (4 waves, 2 per SIMD): kernel A/B + SL bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/tap16
mkdir -p $O
cd $R
VARIANTS=2,5 B=256 timeout -k 10 120 python -u scripts/dbg/conv_ab.py > $O/ab256.json 2> $O/ab256.err || { tail -5 $O/ab256.err; exit 1; }
VARIANTS=2,5 B=512 timeout -k 10 120 python -u scripts/dbg/conv_ab.py > $O/ab512.json 2> $O/ab512.err || exit 1
RAG_CONV_TAP=4 timeout -k 10 200 python -u bench.py --no-mcts > $O/bench4.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --no-mcts > $O/bench1.log 2>&1 || exit 1
cat $O/ab256.json $O/ab512.json; tail -1 $O/bench4.log | cut -c80-160; tail -1 $O/bench1.log | cut -c80-160
