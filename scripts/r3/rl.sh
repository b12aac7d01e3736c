#!/bin/bash
# native self-play test + RL bench (native vs python) + MCTS timeline, 1 GPU
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/rl
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_features.py tests/test_gpu_ladders.py tests/test_gpu_sampling.py tests/test_gpu_models.py tests/test_gpu_search.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for sp in native; do
  timeout -k 10 300 python -u benchmarks/rl_bench.py --config ref7 --selfplay $sp > $O/ref7_$sp.log 2>&1 || { tail -20 $O/ref7_$sp.log; exit 1; }
  grep "^{" $O/ref7_$sp.log
done
for sp in native python; do
  timeout -k 10 400 python -u benchmarks/rl_bench.py --config 19 --game-batch 128 --iterations 1 --selfplay $sp > $O/c19_$sp.log 2>&1 || { tail -20 $O/c19_$sp.log; exit 1; }
  grep "^{" $O/c19_$sp.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o rl -- python3 benchmarks/rl_bench.py --config 19 --game-batch 128 --iterations 1 --selfplay native > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python scripts/dbg/timeline.py $(find $O/prof -name "*.db" | head -1) --window 3 > $O/timeline.txt 2>&1 || true
head -30 $O/timeline.txt
timeout -k 10 300 python -u benchmarks/converter_bench.py --copies 40 --threads 1,4,16 > $O/conv.log 2>&1 || { tail -20 $O/conv.log; exit 1; }
tail -1 $O/conv.log
