#!/bin/bash
# pipelined distributed search: tests, 1-rank and 2-rank (gloo, one GPU) measurements
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/dist2
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_distributed_search.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
timeout -k 10 200 python benchmarks/mcts_bench.py --distributed --moves 4 > $O/mcts_dist1.log 2>&1 || { tail -30 $O/mcts_dist1.log; exit 1; }
RAG_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 benchmarks/mcts_bench.py --distributed --moves 3 --threads 8 > $O/mcts_dist2.log 2>&1
rc=$?
tail -1 $O/tests.log; tail -1 $O/mcts_dist1.log | cut -c1-400; grep sims_per $O/mcts_dist2.log | cut -c1-400
exit $rc
