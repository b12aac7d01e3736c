#!/bin/bash
# wgrad reduce on its own stream (RAG_WGRAD_OVERLAP=1): A/B + kernel trace to see co-residency
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ovl2
mkdir -p $O
cd $R
for rep in 1 2; do
timeout -k 10 200 python -u bench.py --no-mcts --steps 60 > $O/base_$rep.log 2>&1 || exit 1
RAG_WGRAD_OVERLAP=1 timeout -k 10 200 python -u bench.py --no-mcts --steps 60 > $O/ovl_$rep.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
RAG_WGRAD_OVERLAP=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/sl -- python3 $R/bench.py --no-mcts --steps 20 --warmup 3 > $O/sl.log 2>&1 || exit 1
for f in $O/*.log; do echo $(basename $f) $(tail -1 $f | grep -o '"value": [0-9.]*'); done
