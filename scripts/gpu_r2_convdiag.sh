#!/bin/bash
# conv_tap diagnostics (wrong results by design): v6 = no fragment LDS reads, v7 = no waits/barriers/staging, v8 = neither
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/cdiag
cd $R
VARIANTS=2,6,7,8 timeout -k 10 120 python scripts/dbg/conv_ab.py > gpurun_out/cdiag/ab.log 2>&1
rc=$?
tail -1 gpurun_out/cdiag/ab.log
exit $rc
