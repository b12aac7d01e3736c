#!/bin/bash
# 5x5 slab wgrad: kernel tests, SL bench with / without, SL step trace, ResNet bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/w5
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_hip_kernels.py -k "5x5 or backward or wgrad or deferred" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --no-mcts > $O/sl.log 2>&1 || { tail -20 $O/sl.log; exit 1; }
grep "^{" $O/sl.log | cut -c1-200
RAG_WGRAD_SLAB5=0 timeout -k 10 300 python -u bench.py --no-mcts > $O/sl0.log 2>&1 || { tail -20 $O/sl0.log; exit 1; }
grep "^{" $O/sl0.log | cut -c1-200
timeout -k 10 300 python -u bench.py --model resnet --no-mcts > $O/res.log 2>&1 || { tail -20 $O/res.log; exit 1; }
grep "^{" $O/res.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o sl -- python3 bench.py --no-mcts --steps 10 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python scripts/dbg/step_kernels.py $(find $O/prof -name "*.db" | head -1) > $O/step.txt 2>&1 || true
head -16 $O/step.txt
