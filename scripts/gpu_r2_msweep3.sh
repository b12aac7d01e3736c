#!/bin/bash
# wave 512 / 3 in flight: the host waits on rollouts -- hardware queues, rollout streams,
# in-flight limits
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/msweep3
mkdir -p $O
cd $R
run() {
  local n=$1; shift
  env $ENVV timeout -k 10 120 python -u benchmarks/mcts_bench.py --moves 6 "$@" > $O/$n.log 2>&1 || { echo "FAIL $n"; tail -5 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | cut -c1-44) $(tail -1 $O/$n.log | grep -o '"t_rollout_wait_frac": [0-9.]*')"
}
for rep in 1 2; do
ENVV="" run base_$rep
ENVV="GPU_MAX_HW_QUEUES=8" run hwq8_$rep
ENVV="RAG_ROLLOUT_STREAMS=3" run rs3_$rep
ENVV="" run inf16_$rep --max-inflight 16
ENVV="GPU_MAX_HW_QUEUES=8" run hwq8inf16_$rep --max-inflight 16
done
