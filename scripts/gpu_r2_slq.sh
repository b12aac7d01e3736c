#!/bin/bash
# quick SL check: HIP kernel tests, SL bench (no MCTS), one per-step kernel trace. $1 = output tag
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-slq}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py tests/test_gpu_models.py tests/test_pass_logit.py tests/test_gpu_search.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
timeout -k 10 200 python -u bench.py --no-mcts > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/sl -- python3 $R/bench.py --no-mcts --steps 20 --warmup 3 > $O/sl.log 2>&1
rc=$?
tail -1 $O/tests.log; tail -1 $O/bench.log | cut -c1-200
exit $rc
