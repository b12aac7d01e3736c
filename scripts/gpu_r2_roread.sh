#!/bin/bash
# rollout winners read through a pinned copy on the rollout stream: search tests + MCTS A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/roread
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py tests/test_distributed_search.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
run() { n=$1; shift; timeout -k 10 150 python -u benchmarks/mcts_bench.py --moves 6 "$@" > $O/$n.log 2>&1 || exit 1; echo $n $(tail -1 $O/$n.log | cut -c1-400); }
run a1 && run a2 && run lam0 --lmbda 0
tail -1 $O/tests.log
