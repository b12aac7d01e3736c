#!/bin/bash
# 2-rank rehearsal of the bench on ONE GPU over gloo (RCCL needs one GPU per rank): DP training
# with the deferred wgrad reductions + bucket hooks, then the one-search-over-N-GPUs MCTS
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/dp2
mkdir -p $O
cd $R
RAG_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 10 --warmup 3 > $O/bench2.log 2>&1 || { tail -30 $O/bench2.log; exit 1; }
RAG_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 --warmup 3 --model value --no-mcts > $O/bench2v.log 2>&1 || { tail -30 $O/bench2v.log; exit 1; }
grep metric $O/bench2.log | cut -c1-300; grep -o '"mcts[a-z_]*": [^,]*' $O/bench2.log; grep metric $O/bench2v.log | cut -c1-200
