#!/bin/bash
# value-head HIP training kernels: numerics + timing + kernel trace
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_hip_kernels.py -k value_mlp -m gpu > gpurun_out/value_tests.log 2>&1 &&
timeout -k 10 120 python -u scripts/dbg/value_head_time.py > gpurun_out/value_head_time.json 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_vhead -- \
  python3 $R/scripts/dbg/value_head_time.py > $R/gpurun_out/value_head_prof.log 2>&1
rc=$?
cd $R; tail -3 gpurun_out/value_tests.log; cat gpurun_out/value_head_time.json
exit $rc
