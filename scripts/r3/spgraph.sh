#!/bin/bash
# graph-replayed self-play plies: model tests + RL / value-gen benches + RL timeline
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/spgraph
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
run() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1 || { tail -30 $O/$n.log; exit 1; }
  grep "^{" $O/$n.log | tail -1 | cut -c1-700
}
run tests 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_models.py tests/test_gpu_sampling.py
tail -1 $O/tests.log
run c19_native_256 400 python -u benchmarks/rl_bench.py --config 19 --game-batch 256 --iterations 1 --selfplay native
run c19_native_512 400 python -u benchmarks/rl_bench.py --config 19 --game-batch 512 --iterations 1 --selfplay native
run ref7_native 300 python -u benchmarks/rl_bench.py --config ref7 --selfplay native
run vgen_native 400 python -u benchmarks/value_gen_bench.py --games 256 --batch-games 256 --loop native
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o rl -- python3 benchmarks/rl_bench.py --config 19 --game-batch 256 --iterations 1 --selfplay native > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python scripts/dbg/timeline.py $(find $O/prof -name "*.db" | head -1) --window 3 > $O/timeline.txt 2>&1 || true
head -14 $O/timeline.txt
