#!/bin/bash
# host-side options at wave 512: graph-replayed evaluation, async submit
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/hostab
mkdir -p $O
cd $R
for rep in 1; do
for v in both; do
  case $v in
    base) env="" ;;
    graph) env="RAG_EVAL_GRAPH=1" ;;
    async) env="RAG_ASYNC_EVAL=1" ;;
    both) env="RAG_EVAL_GRAPH=1 RAG_ASYNC_EVAL=1" ;;
  esac
  env $env timeout -k 10 120 python -u benchmarks/mcts_bench.py --moves 6 > $O/${v}_$rep.log 2>&1 || { tail -5 $O/${v}_$rep.log; exit 1; }
  echo "${v}_$rep $(tail -1 $O/${v}_$rep.log | cut -c1-48) $(tail -1 $O/${v}_$rep.log | grep -o '"t_submit_frac": [0-9.]*')"
done
done
