#!/bin/bash
# conv kernels: correctness (kernel tests with RAG_CONV_TAP=1/5) + A/B timing + segment diag
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/convpp
mkdir -p $O
cd $R
for m in 8 9; do
RAG_CONV_TAP=$m timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q --timeout 120 --timeout-method thread > $O/tests_m$m.log 2>&1 || { tail -30 $O/tests_m$m.log; exit 1; }
tail -1 $O/tests_m$m.log
done
VARIANTS=2,7,9,10 timeout -k 10 300 python -u scripts/dbg/conv_ab.py > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log | grep "^{"
timeout -k 10 300 python -u scripts/dbg/conv_pp_diag.py > $O/diag.log 2>&1 || { tail -20 $O/diag.log; exit 1; }
grep "^{" $O/diag.log
