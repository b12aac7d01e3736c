#!/bin/bash
# ResnetPolicy SL step: bench + rocprof kernel summary of one step. 1 GPU.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/resprof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 python -u bench.py --model resnet --steps 20 --warmup 5 --no-mcts > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep "^{" $O/bench.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o res -- python3 bench.py --model resnet --steps 8 --warmup 3 --no-mcts > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python scripts/dbg/step_kernels.py $(find $O/prof -name "*.db" | head -1) > $O/step.txt 2>&1 || true
head -40 $O/step.txt
