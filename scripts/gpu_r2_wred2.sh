#!/bin/bash
# wgrad reduce: chunk loads in flight per thread (RAG_WRED_UNROLL) A/B on the SL step + kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/wred2
mkdir -p $O
cd $R
for u in 4 8 16 4 8 16; do
  RAG_WRED_UNROLL=$u timeout -k 10 120 python bench.py --no-mcts --steps 200 --warmup 10 > $O/b$u.log 2>&1 || exit 1
  echo "u=$u $(grep -o '"ms_per_step": [0-9.]*' $O/b$u.log)"
done
for u in 4 8; do
  RAG_WGRAD_OVERLAP=1 RAG_WRED_UNROLL=$u timeout -k 10 120 python bench.py --no-mcts --steps 200 --warmup 10 > $O/o$u.log 2>&1 || exit 1
  echo "overlap u=$u $(grep -o '"ms_per_step": [0-9.]*' $O/o$u.log)"
done
cd /tmp && export TMPDIR=/tmp
for u in 8 16; do
  RAG_WRED_UNROLL=$u timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t$u -- python3 $R/bench.py --no-mcts --steps 20 --warmup 3 > $O/t$u.log 2>&1 || exit 1
done
