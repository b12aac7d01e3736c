#!/bin/bash
# per-step kernel traces of the SL and value training steps (current code)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/steps
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/sl -- python3 $R/bench.py --no-mcts --steps 20 --warmup 3 > $O/sl.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/val -- python3 $R/bench.py --model value --no-mcts --steps 20 --warmup 3 > $O/val.log 2>&1
rc=$?
tail -1 $O/sl.log | cut -c1-120; tail -1 $O/val.log | cut -c1-120
exit $rc
