#!/bin/bash
# wgrad reduction fused into the next dgrad launch: kernel/model tests, A/B, step trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/defer
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py tests/test_gpu_models.py tests/test_resnet_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
for rep in 1 2; do
RAG_WGRAD_DEFER=0 timeout -k 10 200 python -u bench.py --no-mcts --steps 60 > $O/d0_$rep.log 2>&1 || exit 1
RAG_WGRAD_DEFER=1 timeout -k 10 200 python -u bench.py --no-mcts --steps 60 > $O/d1_$rep.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/sl -- python3 $R/bench.py --no-mcts --steps 20 --warmup 3 > $O/sl.log 2>&1 || exit 1
tail -1 $O/tests.log; for f in $O/d*.log; do echo $(basename $f) $(tail -1 $f | grep -o '"value": [0-9.]*'); done
