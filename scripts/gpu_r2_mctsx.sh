#!/bin/bash
# MCTS bound analysis: baseline, no rollouts (lambda 0), bigger rollout groups, more host threads
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/mctsx
mkdir -p $O
cd $R
run() { n=$1; shift; timeout -k 10 150 python -u benchmarks/mcts_bench.py --moves 4 "$@" > $O/$n.log 2>&1 || exit 1; echo $n $(tail -1 $O/$n.log | cut -c1-330); }
run base
run lam0 --lmbda 0
run rg6 --rollout-group 6
run rg6d12 --rollout-group 6 --rollout-delay 12
run thr32 --threads 32
run base2
