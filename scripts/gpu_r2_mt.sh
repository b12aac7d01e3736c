#!/bin/bash
# 5x5 conv tile choice at B=512 (MCTS waves): kernel timing + MCTS bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/mt
mkdir -p $O
cd $R
B=512 VARIANTS=2 timeout -k 10 120 python scripts/dbg/conv_ab.py > $O/ab512.log 2>&1 || { tail -5 $O/ab512.log; exit 1; }
tail -1 $O/ab512.log
for rep in 1 2; do
timeout -k 10 120 python -u benchmarks/mcts_bench.py --moves 6 > $O/mcts_$rep.log 2>&1 || exit 1
tail -1 $O/mcts_$rep.log | cut -c1-60
done
