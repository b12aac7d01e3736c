#!/bin/bash
# 192-pixel 5x5 ping-pong blocks: conv tests, B=128 conv A/B, RL / value-gen
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pp192c
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv_forward or conv_backward or pingpong" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 1 0; do
  RAG_CONV_PP5=$v B=128 VARIANTS=7 timeout -k 10 120 python -u scripts/dbg/conv_ab.py > $O/ab128_$v.json 2>&1 || { tail -20 $O/ab128_$v.json; exit 1; }
  echo "B128 PP5=$v $(tail -1 $O/ab128_$v.json)"
done
timeout -k 10 240 python -u benchmarks/rl_bench.py --config 19 --game-batch 256 --iterations 1 > $O/rl.log 2>&1 || { tail -20 $O/rl.log; exit 1; }
echo "$(tail -1 $O/rl.log | cut -c 200-)"
timeout -k 10 240 python -u benchmarks/value_gen_bench.py > $O/vgen.log 2>&1 || { tail -20 $O/vgen.log; exit 1; }
tail -1 $O/vgen.log
