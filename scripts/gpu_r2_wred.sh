#!/bin/bash
# wgrad reduce with 16 loads in flight: numerics, SL bench, kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/wred
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py tests/test_gpu_models.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
timeout -k 10 200 python -u bench.py --no-mcts > $O/bench.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $R/bench.py --no-mcts --steps 20 --warmup 3 > $O/prof.log 2>&1
rc=$?
cd $R; tail -1 $O/tests.log; tail -1 $O/bench.log | cut -c1-200
exit $rc
