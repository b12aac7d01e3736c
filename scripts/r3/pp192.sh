#!/bin/bash
# 192-pixel ping-pong blocks for sub-chip grids: conv tests, B=128 conv A/B, RL / value-gen A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pp192
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv_forward or conv_backward" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 1 0; do
  RAG_CONV_PP192=$v B=128 VARIANTS=7 timeout -k 10 120 python -u scripts/dbg/conv_ab.py > $O/ab_$v.json 2>&1 || { tail -20 $O/ab_$v.json; exit 1; }
  echo "pp192=$v $(tail -1 $O/ab_$v.json)"
done
for v in 1 0; do
  RAG_CONV_PP192=$v timeout -k 10 240 python -u benchmarks/rl_bench.py --config 19 --game-batch 256 --iterations 1 > $O/rl_$v.log 2>&1 || { tail -20 $O/rl_$v.log; exit 1; }
  echo "pp192=$v $(tail -1 $O/rl_$v.log | cut -c 200-)"
done
RAG_CONV_PP192=1 timeout -k 10 240 python -u benchmarks/value_gen_bench.py > $O/vgen.log 2>&1 || { tail -20 $O/vgen.log; exit 1; }
tail -1 $O/vgen.log
