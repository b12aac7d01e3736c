#!/bin/bash
# round 3: packed-wave search path — GPU search tests, then MCTS bench (packed vs board path,
# graph on/off) and the null-evaluator host ceiling on the box's CPUs
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/mcts1
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for cfg in "RAG_PACKED_WAVES=0" "RAG_PACKED_WAVES=1" "RAG_PACKED_WAVES=1 RAG_EVAL_GRAPH=1"; do
  echo "== $cfg" >> $O/bench.log
  env $cfg timeout -k 10 200 python -u benchmarks/mcts_bench.py --moves 4 >> $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
done
grep -v "^==" $O/bench.log | cut -c1-400
timeout -k 10 200 python -u benchmarks/mcts_null_bench.py --threads 16 --playouts 65536 > $O/null.log 2>&1 || exit 1
cat $O/null.log
