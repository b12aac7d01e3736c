#!/bin/bash
# value-net training bench + kernel stats (value head now on value_bwd.hip)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u bench.py --model value --no-mcts --steps 30 --warmup 5 \
  > gpurun_out/value_bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_value -o run -- \
  python3 bench.py --model value --no-mcts --steps 10 --warmup 3 > gpurun_out/value_prof.log 2>&1
rc=$?
tail -3 gpurun_out/value_bench.log
exit $rc
