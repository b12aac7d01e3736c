#!/bin/bash
# full GPU suite, smoke, headline bench (SL + MCTS), value + resnet benches, SL step kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/full
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
timeout -k 10 200 python -u bench.py --model value --no-mcts > $O/bench_value.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --model resnet --no-mcts > $O/bench_resnet.log 2>&1 || exit 1
for f in bench bench_value bench_resnet; do tail -1 $O/$f.log | cut -c1-400; done
grep -o '"mcts_sims_per_s": [0-9.]*' $O/bench.log
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o sl -- python3 bench.py --no-mcts --steps 10 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
