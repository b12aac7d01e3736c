#!/bin/bash
# round-end rehearsal: full GPU suite, smoke, headline bench (SL + MCTS), value and resnet benches
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/end
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
timeout -k 10 200 python -u bench.py --model value --no-mcts > $O/bench_value.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --model resnet --no-mcts > $O/bench_resnet.log 2>&1 || exit 1
tail -2 $O/gpu_tests.log; tail -1 $O/smoke.log
for f in bench bench_value bench_resnet; do tail -1 $O/$f.log | cut -c1-150; done
grep -o '"mcts_sims_per_s": [0-9.]*' $O/bench.log
