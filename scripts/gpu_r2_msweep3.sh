#!/bin/bash
# wave 512 / 3 in flight: rollout grouping and in-flight limits (the host waits on rollouts)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/msweep3
mkdir -p $O
cd $R
run() {
  local n=$1; shift
  timeout -k 10 120 python -u benchmarks/mcts_bench.py --moves 6 "$@" > $O/$n.log 2>&1 || { echo "FAIL $n"; tail -5 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | cut -c1-44) $(tail -1 $O/$n.log | grep -o '"t_rollout_wait_frac": [0-9.]*')"
}
for rep in 1 2; do
run base_$rep
run inf16_$rep --max-inflight 16
run inf24_$rep --max-inflight 24
run g2inf16_$rep --rollout-group 2 --max-inflight 16
run g1inf16_$rep --rollout-group 1 --max-inflight 16
done
