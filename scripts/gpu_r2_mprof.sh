#!/bin/bash
# MCTS kernel stats at the current defaults (wave 512, 3 in flight)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/mprof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $R/benchmarks/mcts_bench.py --moves 3 > $O/prof.log 2>&1
rc=$?
tail -1 $O/prof.log | cut -c1-300
exit $rc
