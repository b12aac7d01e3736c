#!/bin/bash
# CU partition for search rollouts: A/B over RAG_ROLLOUT_CU_ROUNDS, timeline at 2 rounds
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/cumask
mkdir -p $O
RAG_ROLLOUT_CU_ROUNDS=2 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  $R/tests/test_gpu_search.py -m gpu > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
for r in 0 1 2 3; do
  RAG_ROLLOUT_CU_ROUNDS=$r timeout -k 10 200 python -u $R/benchmarks/mcts_bench.py --moves 6 > $O/mcts_r$r.log 2>&1 || { tail -20 $O/mcts_r$r.log; exit 1; }
done
cd /tmp && export TMPDIR=/tmp &&
RAG_ROLLOUT_CU_ROUNDS=2 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof -- \
  python3 $R/benchmarks/mcts_bench.py --moves 2 > $O/prof.log 2>&1
rc=$?
cd $R; tail -1 $O/tests.log; for r in 0 1 2 3; do echo r$r; tail -1 $O/mcts_r$r.log | cut -c1-330; done
exit $rc
