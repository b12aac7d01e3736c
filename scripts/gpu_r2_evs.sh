#!/bin/bash
# search GPU tests + A/B of two-stream leaf evaluation (RAG_EVAL_STREAMS=2), rollout group 6
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/evs
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
run() { n=$1; e=$2; shift 2; env $e timeout -k 10 150 python -u benchmarks/mcts_bench.py --moves 6 "$@" > $O/$n.log 2>&1 || exit 1; echo $n $(tail -1 $O/$n.log | cut -c1-60); }
for rep in 1 2; do
run one_$rep RAG_EVAL_STREAMS=1
run two_$rep RAG_EVAL_STREAMS=2
done
run lam0one RAG_EVAL_STREAMS=1 --lmbda 0
tail -1 $O/tests.log
