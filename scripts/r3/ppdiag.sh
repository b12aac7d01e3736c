#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ppdiag
mkdir -p $O
cd $R
timeout -k 10 300 python -u scripts/dbg/conv_pp_diag.py > $O/diag.log 2>&1 || { tail -20 $O/diag.log; exit 1; }
B=512 timeout -k 10 300 python -u scripts/dbg/conv_pp_diag.py >> $O/diag.log 2>&1 || { tail -20 $O/diag.log; exit 1; }
grep "^{" $O/diag.log
