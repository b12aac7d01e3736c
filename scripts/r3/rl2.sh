#!/bin/bash
# GPU tests (features / models / resnet / pass logit / search) + RL and value-gen benches,
# SL bench regression check, RL kernel timeline. 1 GPU.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/rl2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_models.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for G in 256; do
  timeout -k 10 400 python -u benchmarks/rl_bench.py --config 19 --game-batch $G --iterations 1 --selfplay native > $O/c19_$G.log 2>&1 || { tail -20 $O/c19_$G.log; exit 1; }
  grep "^{" $O/c19_$G.log
done
for L in native python; do
  timeout -k 10 400 python -u benchmarks/value_gen_bench.py --games 128 --batch-games 128 --loop $L > $O/vgen_$L.log 2>&1 || { tail -20 $O/vgen_$L.log; exit 1; }
  grep "^{" $O/vgen_$L.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o rl -- python3 benchmarks/rl_bench.py --config 19 --game-batch 256 --iterations 1 --selfplay native > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python scripts/dbg/timeline.py $(find $O/prof -name "*.db" | head -1) --window 3 > $O/timeline.txt 2>&1 || true
head -30 $O/timeline.txt
timeout -k 10 300 python -u benchmarks/converter_bench.py --copies 40 --threads 1,4,16 > $O/conv.log 2>&1 || { tail -20 $O/conv.log; exit 1; }
tail -1 $O/conv.log
