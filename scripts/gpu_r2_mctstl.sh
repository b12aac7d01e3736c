#!/bin/bash
# MCTS bench + kernel timeline (for GPU-occupancy analysis of the search)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/mctstl
timeout -k 10 200 python -u $R/benchmarks/mcts_bench.py --moves 2 > $R/gpurun_out/mctstl/bench.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/mctstl/prof -- \
  python3 $R/benchmarks/mcts_bench.py --moves 2 > $R/gpurun_out/mctstl/prof.log 2>&1
rc=$?
tail -2 $R/gpurun_out/mctstl/bench.log
exit $rc
