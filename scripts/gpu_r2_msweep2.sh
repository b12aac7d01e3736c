#!/bin/bash
# MCTS wave size / pipeline depth, repeated (run-to-run noise is ~+-5 %)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/msweep2
mkdir -p $O
cd $R
run() {
  local n=$1; shift
  timeout -k 10 120 python -u benchmarks/mcts_bench.py --moves 6 "$@" > $O/$n.log 2>&1 || { echo "FAIL $n"; tail -5 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | cut -c1-48)"
}
for rep in 1 2; do
run base_$rep
run b512_$rep --batch 512
run b512p3_$rep --batch 512 --pipeline 3
run b768_$rep --batch 768
done
timeout -k 10 200 python benchmarks/converter_bench.py --copies 40 --threads 1,4,16 > $O/conv.log 2>&1 && echo "conv $(tail -1 $O/conv.log)"
