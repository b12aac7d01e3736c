#!/bin/bash
# APV-MCTS leaf-wave size: 512 vs 544 (a B = 544 trunk conv is 1023 blocks = two full block waves)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/wave
mkdir -p $O
cd $R
run() { n=$1; shift; timeout -k 10 150 python -u benchmarks/mcts_bench.py --moves 6 "$@" > $O/$n.log 2>&1 || exit 1; echo $n $(tail -1 $O/$n.log | cut -c1-60); }
for rep in 1 2; do
run b512_$rep --batch 512
run b544_$rep --batch 544
run b480_$rep --batch 480
done
