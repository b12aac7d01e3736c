#!/bin/bash
# graph-replayed leaf evaluation: tests, then MCTS bench A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/graph
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  $R/tests/test_gpu_search.py $R/tests/test_apv.py -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
for rep in 1 2; do
for gr in 1 0; do
  RAG_EVAL_GRAPH=$gr timeout -k 10 200 python -u $R/benchmarks/mcts_bench.py --moves 6 > $O/mcts_g${gr}_$rep.log 2>&1 || { grep -v "^frame" $O/mcts_g${gr}_$rep.log | tail -20; exit 1; }
done
done
tail -2 $O/tests.log; for f in $O/mcts_g*.log; do echo $f; tail -1 $f | cut -c1-330; done
