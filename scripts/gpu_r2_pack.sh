#!/bin/bash
# tiled pack_trunk: GPU tests touching the trunk + SL step kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pack
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_kernels.py tests/test_gpu_models.py > $O/tests.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/sl -- python3 $R/bench.py --no-mcts --steps 20 --warmup 3 > $O/sl.log 2>&1
rc=$?
tail -2 $O/tests.log; tail -1 $O/sl.log | cut -c1-160
exit $rc
