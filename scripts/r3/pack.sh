#!/bin/bash
# repack / input-pack kernels: tests, SL bench, SL step kernel stats, RL GPU-busy share
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pack
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py tests/test_gpu_models.py -m gpu -x -q --timeout 120 --timeout-method thread -k "pack or repack or train_step or value" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python -u bench.py --no-mcts > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o sl -- python3 bench.py --no-mcts --steps 10 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/dbg/step_kernels.py $(find $O/prof -name "*.db" | head -1) > $O/step.txt 2>&1 || true
timeout -k 10 240 python -u benchmarks/rl_bench.py --config 19 --game-batch 256 --iterations 1 > $O/rl_256.log 2>&1 || { tail -20 $O/rl_256.log; exit 1; }
tail -1 $O/rl_256.log
