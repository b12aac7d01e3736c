#!/bin/bash
# 192-pixel ping-pong blocks at 2 blocks per CU: B=128 and B=256 conv A/B, SL bench A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pp192b
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv_forward or conv_backward" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
RAG_CONV_PP192=1 B=128 VARIANTS=7 timeout -k 10 120 python -u scripts/dbg/conv_ab.py > $O/ab128.json 2>&1 || { tail -20 $O/ab128.json; exit 1; }
echo "B128 pp192 $(tail -1 $O/ab128.json)"
for v in 1 2; do
  RAG_CONV_PP192=$v B=256 VARIANTS=7 timeout -k 10 120 python -u scripts/dbg/conv_ab.py > $O/ab256_$v.json 2>&1 || { tail -20 $O/ab256_$v.json; exit 1; }
  echo "B256 PP192=$v $(tail -1 $O/ab256_$v.json)"
done
for v in 1 2; do
  RAG_CONV_PP192=$v timeout -k 10 200 python -u bench.py --no-mcts > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  echo "PP192=$v $(tail -1 $O/bench_$v.log | cut -c1-200)"
done
