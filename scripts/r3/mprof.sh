#!/bin/bash
# APV-MCTS kernel timeline (GPU busy fraction) + host phase split, 1 GPU
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/mprof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 python -u benchmarks/mcts_bench.py --moves 6 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep "^{" $O/bench.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o mcts -- python3 benchmarks/mcts_bench.py --moves 4 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python scripts/dbg/timeline.py $(find $O/prof -name "*.db" | head -1) --window 0.25 > $O/timeline.txt
cat $O/timeline.txt | head -30
