#!/bin/bash
# RL self-play / training + value-data generation throughput (native lock-step engine vs the
# per-game Python loop), RL kernel timeline, converter thread scaling. 1 GPU.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/rlprof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
run() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  grep "^{" $O/$n.log | tail -1 | cut -c1-600
}
run ref7_native 300 python -u benchmarks/rl_bench.py --config ref7 --selfplay native
run ref7_python 300 python -u benchmarks/rl_bench.py --config ref7 --selfplay python
run c19_native_256 400 python -u benchmarks/rl_bench.py --config 19 --game-batch 256 --iterations 1 --selfplay native
run c19_python_64 400 python -u benchmarks/rl_bench.py --config 19 --game-batch 64 --iterations 1 --selfplay python
run c19_native_64 400 python -u benchmarks/rl_bench.py --config 19 --game-batch 64 --iterations 1 --selfplay native
run vgen_native 400 python -u benchmarks/value_gen_bench.py --games 256 --batch-games 256 --loop native
run vgen_python 400 python -u benchmarks/value_gen_bench.py --games 128 --batch-games 128 --loop python
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o rl -- python3 benchmarks/rl_bench.py --config 19 --game-batch 256 --iterations 1 --selfplay native > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python scripts/dbg/timeline.py $(find $O/prof -name "*.db" | head -1) --window 3 > $O/timeline.txt 2>&1 || true
head -30 $O/timeline.txt
run conv 300 python -u benchmarks/converter_bench.py --copies 40 --threads 1,4,16
