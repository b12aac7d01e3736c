#!/bin/bash
# rollout kernel: bit-exact tests, standalone throughput at both register budgets, MCTS bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ro2
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  $R/tests/test_gpu_search.py -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
for wpe in 4 3; do
RAG_ROLLOUT_WPE=$wpe timeout -k 10 120 python -u $R/benchmarks/rollout_bench.py > $O/rollout_wpe$wpe.jsonl 2>&1 || exit 1
done
timeout -k 10 200 python -u $R/benchmarks/mcts_bench.py --moves 6 > $O/mcts.log 2>&1
rc=$?
tail -1 $O/tests.log; grep -h games $O/rollout_wpe*.jsonl; tail -1 $O/mcts.log | cut -c1-300
exit $rc
