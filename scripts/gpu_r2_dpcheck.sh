#!/bin/bash
# DP replica identity on the HIP training path: 2 ranks on one GPU over gloo; default kernels and
# fp32 partial slabs without deferral (bf16-noise baseline of the single-process comparison)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/dpcheck
mkdir -p $O
cd $R
run() { n=$1; shift; env RAG_DIST_BACKEND=gloo "$@" timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29631 scripts/dbg/dp_replica_check.py > $O/$n.log 2>&1; rc=$?; echo $n $(grep -E '^\{' $O/$n.log); return $rc; }
run default && run fp32part_nodefer RAG_WGRAD_PART=fp32 RAG_WGRAD_DEFER=0
