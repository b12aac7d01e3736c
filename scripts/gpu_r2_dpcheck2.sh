#!/bin/bash
# DP vs single-process update difference after 1 and 4 steps (fp16 and fp32 partials)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/dpcheck2
mkdir -p $O
cd $R
run() { n=$1; shift; env RAG_DIST_BACKEND=gloo "$@" timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29631 scripts/dbg/dp_replica_check.py > $O/$n.log 2>&1; rc=$?; echo $n $(grep -E '^\{' $O/$n.log); return $rc; }
run s1_fp16 DP_CHECK_STEPS=1 && run s1_fp32 DP_CHECK_STEPS=1 RAG_WGRAD_PART=fp32 && run s2_fp16 DP_CHECK_STEPS=2
