#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 120 python $R/scripts/dbg/gemm_ref.py > $R/gpurun_out/gemm_ref.json 2>&1
rc=$?
tail -2 $R/gpurun_out/gemm_ref.json
exit $rc
