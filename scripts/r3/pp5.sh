#!/bin/bash
# 5x5 ping-pong conv: kernel + model tests, SL and ResNet benches with / without, SL step trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pp5
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_hip_kernels.py tests/test_resnet_gpu.py tests/test_gpu_models.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 1 0; do
  RAG_CONV_PP5=$v timeout -k 10 300 python -u bench.py --no-mcts > $O/sl$v.log 2>&1 || { tail -20 $O/sl$v.log; exit 1; }
  grep "^{" $O/sl$v.log | cut -c1-170
  RAG_CONV_PP5=$v timeout -k 10 300 python -u bench.py --model resnet --no-mcts > $O/res$v.log 2>&1 || { tail -20 $O/res$v.log; exit 1; }
  grep "^{" $O/res$v.log | cut -c1-170
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o sl -- python3 bench.py --no-mcts --steps 10 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python scripts/dbg/step_kernels.py $(find $O/prof -name "*.db" | head -1) > $O/step.txt 2>&1 || true
head -12 $O/step.txt
