#!/bin/bash
# BN backward finalize folded into the apply: tests, ResNet bench A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/bnfold
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_resnet_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
  for v in 1 0; do
    RAG_BN_FOLD=$v timeout -k 10 200 python -u bench.py --model resnet --no-mcts > $O/res_${v}_$rep.log 2>&1 || { tail -20 $O/res_${v}_$rep.log; exit 1; }
    echo "FOLD=$v rep $rep: $(tail -1 $O/res_${v}_$rep.log | cut -c1-160)"
  done
done
