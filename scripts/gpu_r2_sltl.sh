#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/sltl
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof -- python3 $R/bench.py --no-mcts --steps 20 --warmup 3 > $O/prof.log 2>&1
rc=$?
tail -1 $O/prof.log | cut -c1-200
exit $rc
