#!/bin/bash
# conv_tap A/B: variant 2 = mode 1 (current), 5 = mode 4 (slab fragments read before the barrier)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/cab3
cd $R
VARIANTS=2,5 timeout -k 10 120 python scripts/dbg/conv_ab.py > gpurun_out/cab3/ab.log 2>&1
rc=$?
tail -5 gpurun_out/cab3/ab.log
exit $rc
