#!/bin/bash
# bf16 wgrad partial slabs + per-(pixel, 8-channel) input packing: kernel tests, bench, step trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/bfpart
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py tests/test_gpu_models.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
RAG_WGRAD_PART=fp32 timeout -k 10 200 python -u bench.py --no-mcts > $O/bench_fp32part.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/sl -- python3 $R/bench.py --no-mcts --steps 20 --warmup 3 > $O/sl.log 2>&1
rc=$?
tail -2 $O/tests.log; tail -1 $O/bench.log | cut -c1-200; tail -1 $O/bench_fp32part.log | cut -c1-200
exit $rc
