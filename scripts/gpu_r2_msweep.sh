#!/bin/bash
# MCTS knob sweep after the rollout-kernel speedup
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/msweep
mkdir -p $O
cd $R
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 120 python -u benchmarks/mcts_bench.py --moves 4 "$@" > $O/$n.log 2>&1 || { echo "FAIL $n"; tail -5 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | cut -c1-60)"
}
run base
run g2 --rollout-group 2
run g4 --rollout-group 4
run g6 --rollout-group 6
run inf12 --max-inflight 12
run p3 --pipeline 3
run b384 --batch 384
run b512 --batch 512
run base2
timeout -k 10 200 python -u bench.py --model resnet --no-mcts > $O/resnet.log 2>&1 && echo "resnet $(tail -1 $O/resnet.log | cut -c1-140)"
timeout -k 10 300 python benchmarks/converter_bench.py --copies 40 --threads 1,4,16 > $O/conv.log 2>&1 && echo "conv $(tail -1 $O/conv.log)"
