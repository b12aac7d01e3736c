#!/bin/bash
# rollout GPB A/B with longer runs (alternating), and a no-rollout (lambda 0) timeline
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/gpb2
mkdir -p $O
for rep in 1 2; do
for g in 4 1; do
  RAG_ROLLOUT_GPB=$g timeout -k 10 200 python -u $R/benchmarks/mcts_bench.py --moves 6 > $O/mcts_gpb${g}_$rep.log 2>&1 || exit 1
done
done
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof0 -- \
  python3 $R/benchmarks/mcts_bench.py --moves 2 --lmbda 0 > $O/prof0.log 2>&1
rc=$?
cd $R; for f in $O/mcts_gpb*.log; do echo $f; tail -1 $f | cut -c1-330; done
exit $rc
