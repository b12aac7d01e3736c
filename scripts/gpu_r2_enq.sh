#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 200 python -u $R/scripts/dbg/host_enqueue.py > $R/gpurun_out/host_enqueue.log 2>&1
rc=$?
tail -5 $R/gpurun_out/host_enqueue.log
exit $rc
