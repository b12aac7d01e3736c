#!/bin/bash
# round 3: packed-wave search path + exact-bench-path parity tests, MCTS bench A/B (packed vs
# board path, graph on/off), null-evaluator host ceiling on the box's CPUs
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/mcts1
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_bench_path.py -x -v -s --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
grep -E "rel. error|PASS|FAIL|passed|failed" $O/tests.log | cut -c1-600
for cfg in "RAG_PACKED_WAVES=0" "RAG_PACKED_WAVES=1" "RAG_PACKED_WAVES=1 RAG_EVAL_GRAPH=1"; do
  echo "== $cfg" >> $O/bench.log
  env $cfg timeout -k 10 200 python -u benchmarks/mcts_bench.py --moves 4 >> $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
done
grep -v "^==" $O/bench.log | cut -c1-400
for t in 4 16 32; do
timeout -k 10 200 python -u benchmarks/mcts_null_bench.py --threads $t --playouts 65536 >> $O/null.log 2>&1 || exit 1
done
cat $O/null.log
