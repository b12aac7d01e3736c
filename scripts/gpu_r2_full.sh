#!/bin/bash
# full GPU suite + smoke + bench (round-end rehearsal)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/full
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1
rc=$?
tail -2 $O/gpu_tests.log; tail -2 $O/smoke.log; tail -1 $O/bench.log
exit $rc
