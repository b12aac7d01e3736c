#!/bin/bash
# A/B: wgrad reduction on its own stream (RAG_WGRAD_OVERLAP=1) vs in-stream, bf16 partials
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ovl
mkdir -p $O
cd $R
for i in 1 2; do
timeout -k 10 200 python -u bench.py --no-mcts --steps 60 > $O/base_$i.log 2>&1 || exit 1
RAG_WGRAD_OVERLAP=1 timeout -k 10 200 python -u bench.py --no-mcts --steps 60 > $O/ovl_$i.log 2>&1 || exit 1
done
for f in $O/*.log; do echo $(basename $f) $(tail -1 $f | cut -c80-150); done
