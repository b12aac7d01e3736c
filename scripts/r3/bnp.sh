#!/bin/bash
# BN prologue fusion: ResNet tests + kernel tests, ResNet bench, ResNet step trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/bnp
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_resnet_gpu.py tests/test_hip_kernels.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench.py --model resnet --steps 20 --warmup 5 --no-mcts > $O/bench_res.log 2>&1 || { tail -20 $O/bench_res.log; exit 1; }
grep "^{" $O/bench_res.log | cut -c1-300
RAG_BN_PROLOGUE=0 timeout -k 10 300 python -u bench.py --model resnet --steps 20 --warmup 5 --no-mcts > $O/bench_res0.log 2>&1 || { tail -20 $O/bench_res0.log; exit 1; }
grep "^{" $O/bench_res0.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o res -- python3 bench.py --model resnet --steps 8 --warmup 3 --no-mcts > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python scripts/dbg/step_kernels.py $(find $O/prof -name "*.db" | head -1) > $O/step.txt 2>&1 || true
head -30 $O/step.txt
