#!/bin/bash
# ping-pong wgrad: kernel tests, A/B timing, SL bench with/without, SL step trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/wpp
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_hip_kernels.py -k "wgrad or deferred" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u scripts/dbg/wgrad_pp_ab.py > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
tail -1 $O/ab.log
timeout -k 10 300 python -u bench.py --no-mcts > $O/sl_pp.log 2>&1 || { tail -20 $O/sl_pp.log; exit 1; }
grep "^{" $O/sl_pp.log | cut -c1-200
RAG_WGRAD_PP=0 timeout -k 10 300 python -u bench.py --no-mcts > $O/sl_nopp.log 2>&1 || { tail -20 $O/sl_nopp.log; exit 1; }
grep "^{" $O/sl_nopp.log | cut -c1-200
