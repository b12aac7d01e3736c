#!/bin/bash
# RL self-play: GPU busy share of the pipelined ply loop (selfplay_gpu_busy), game batch 256 / 512
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/rlbusy
mkdir -p $O
cd $R
for g in 256 512; do
  timeout -k 10 240 python -u benchmarks/rl_bench.py --config 19 --game-batch $g --iterations 1 > $O/rl_$g.log 2>&1 || { tail -20 $O/rl_$g.log; exit 1; }
  tail -1 $O/rl_$g.log
done
timeout -k 10 240 python -u benchmarks/value_gen_bench.py > $O/vgen.log 2>&1 || { tail -20 $O/vgen.log; exit 1; }
tail -1 $O/vgen.log
