#!/bin/bash
# MCTS: 384-pixel conv blocks (default) vs 192-pixel blocks everywhere (RAG_CONV_PP192=2) at waves of 512
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/wave2
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in 1 2; do
    RAG_CONV_PP192=$v timeout -k 10 200 python -u benchmarks/mcts_bench.py --moves 6 > $O/mcts_${v}_$rep.log 2>&1 || { tail -20 $O/mcts_${v}_$rep.log; exit 1; }
    echo "PP192=$v rep $rep: $(tail -1 $O/mcts_${v}_$rep.log | cut -c1-120)"
  done
done
