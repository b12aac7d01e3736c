#!/bin/bash
# after the cheap stream-handle fix: RL self-play, value gen, MCTS, SL bench + GPU tests
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/hostfix
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
run() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  grep "^{" $O/$n.log | tail -1 | cut -c1-700
}
run gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
tail -1 $O/gpu_tests.log
run c19_native_256 400 python -u benchmarks/rl_bench.py --config 19 --game-batch 256 --iterations 1 --selfplay native
run c19_native_512 400 python -u benchmarks/rl_bench.py --config 19 --game-batch 512 --iterations 1 --selfplay native
run ref7_native 300 python -u benchmarks/rl_bench.py --config ref7 --selfplay native
run vgen_native 400 python -u benchmarks/value_gen_bench.py --games 256 --batch-games 256 --loop native
run mcts 300 python -u benchmarks/mcts_bench.py --moves 6
run sl 300 python -u bench.py
