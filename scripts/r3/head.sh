#!/bin/bash
# policy head forward at 384 threads: head/model tests, SL step kernel stats, bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/head
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py tests/test_gpu_models.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o sl -- python3 bench.py --no-mcts --steps 10 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/dbg/step_kernels.py $(find $O/prof -name "*.db" | head -1) > $O/step.txt 2>&1
grep -i "head\|step" $O/step.txt
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
grep -o '"mcts_sims_per_s": [0-9.]*' $O/bench.log
