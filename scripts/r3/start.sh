#!/bin/bash
# round-3 start: GPU suite, smoke, headline bench on the unchanged round-2 tree
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3start
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -2 $O/gpu_tests.log; tail -1 $O/bench.log
