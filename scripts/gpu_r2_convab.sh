#!/bin/bash
# conv_tap A/B: variant 2 = conv_tap (mode 1), 3 = conv_deep (mode 2)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/cab4
cd $R
VARIANTS=2,3 timeout -k 10 120 python scripts/dbg/conv_ab.py > gpurun_out/cab4/ab.log 2>&1
rc=$?
tail -5 gpurun_out/cab4/ab.log
exit $rc
