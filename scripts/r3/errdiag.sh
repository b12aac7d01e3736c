#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/errdiag
mkdir -p $O
cd $R
for cfg in "L=12" "L=12 RAG_WGRAD_PART=fp32" "L=12 RAG_WGRAD_DEFER=0 RAG_WGRAD_PART=fp32" "L=3" "L=12 B=64"; do
  env $cfg timeout -k 10 120 python -u scripts/dbg/bench_path_err.py >> $O/err.log 2>&1 || { tail -20 $O/err.log; exit 1; }
done
cat $O/err.log | grep "^{"
