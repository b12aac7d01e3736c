#!/bin/bash
# ResnetPolicy step kernel breakdown (current tree)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/resprof2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o res -- python3 bench.py --model resnet --no-mcts --steps 10 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/dbg/step_kernels.py $(find $O/prof -name "*.db" | head -1) > $O/step.txt 2>&1
cat $O/step.txt
