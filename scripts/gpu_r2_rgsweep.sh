#!/bin/bash
# rollout launch grouping x rollout waves in flight (APV-MCTS, wave 512, 3 in flight, --moves 6)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/rgsweep
mkdir -p $O
cd $R
run() { n=$1; shift; timeout -k 10 150 python -u benchmarks/mcts_bench.py --moves 6 "$@" > $O/$n.log 2>&1 || exit 1; echo $n $(tail -1 $O/$n.log | cut -c1-60); }
for rep in 1 2; do
run rg3i8_$rep --rollout-group 3 --max-inflight 8
run rg6i8_$rep --rollout-group 6 --max-inflight 8
run rg6i12_$rep --rollout-group 6 --max-inflight 12
run rg8i16_$rep --rollout-group 8 --max-inflight 16
run rg4i8_$rep --rollout-group 4 --max-inflight 8
done
