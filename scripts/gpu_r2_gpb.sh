#!/bin/bash
# rollout games-per-block A/B: standalone rollouts, MCTS bench, timeline with GPB=1
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/gpb
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  $R/tests/test_gpu_search.py -m gpu -k rollout > $O/tests.log 2>&1 &&
for g in 4 1; do
  RAG_ROLLOUT_GPB=$g timeout -k 10 120 python -u $R/benchmarks/rollout_bench.py > $O/rollout_gpb$g.jsonl 2>&1 || exit 1
  RAG_ROLLOUT_GPB=$g timeout -k 10 200 python -u $R/benchmarks/mcts_bench.py --moves 3 > $O/mcts_gpb$g.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp &&
RAG_ROLLOUT_GPB=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof -- \
  python3 $R/benchmarks/mcts_bench.py --moves 2 > $O/prof.log 2>&1
rc=$?
cd $R; tail -1 $O/tests.log; for g in 4 1; do cat $O/rollout_gpb$g.jsonl | grep games; tail -1 $O/mcts_gpb$g.log | cut -c1-200; done
exit $rc
