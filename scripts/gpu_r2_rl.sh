#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  $R/tests/test_gpu_models.py -m gpu > $R/gpurun_out/rl_tests.log 2>&1
rc=$?
tail -15 $R/gpurun_out/rl_tests.log
exit $rc
