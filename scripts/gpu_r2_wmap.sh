#!/bin/bash
# wgrad_slab wave->tile map A/B (RAG_WGRAD_MAP 0: 2 n x 9 taps per wave, 1: 6 n x 3 taps) + step trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/wmap
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
for rep in 1 2; do
RAG_WGRAD_MAP=0 timeout -k 10 200 python -u bench.py --no-mcts --steps 60 > $O/m0_$rep.log 2>&1 || exit 1
RAG_WGRAD_MAP=1 timeout -k 10 200 python -u bench.py --no-mcts --steps 60 > $O/m1_$rep.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/sl -- python3 $R/bench.py --no-mcts --steps 20 --warmup 3 > $O/sl.log 2>&1 || exit 1
tail -1 $O/tests.log; for f in $O/m*.log; do echo $(basename $f) $(tail -1 $f | grep -o '"value": [0-9.]*'); done
