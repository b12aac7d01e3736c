#!/bin/bash
# MCTS wave size A/B: 512 leaves (482 conv blocks of 384 px: 1.88 rounds on 256 CUs) vs 544 (512 blocks)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/wave
mkdir -p $O
cd $R
for rep in 1 2; do
  for b in 512 544; do
    timeout -k 10 200 python -u benchmarks/mcts_bench.py --moves 6 --batch $b > $O/mcts_${b}_$rep.log 2>&1 || { tail -20 $O/mcts_${b}_$rep.log; exit 1; }
    echo "batch $b rep $rep: $(tail -1 $O/mcts_${b}_$rep.log | cut -c1-300)"
  done
done
