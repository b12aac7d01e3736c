#!/bin/bash
# GPU suite + cProfile of one RL self-play iteration (19x19, G=256) + RL bench at G=512
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/spprof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -u -m cProfile -s tottime benchmarks/rl_bench.py --config 19 --game-batch 256 --iterations 1 --selfplay native > $O/cprof.log 2>&1 || { tail -20 $O/cprof.log; exit 1; }
grep "^{" $O/cprof.log | cut -c1-400
grep -A45 "Ordered by" $O/cprof.log | head -50
timeout -k 10 400 python -u benchmarks/rl_bench.py --config 19 --game-batch 512 --iterations 1 --selfplay native > $O/c19_512.log 2>&1 || { tail -20 $O/c19_512.log; exit 1; }
grep "^{" $O/c19_512.log | cut -c1-600
