#!/bin/bash
# rehearse the driver's N>1 bench path with 2 ranks on one GPU (gloo; the driver uses RCCL on 8 GPUs)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/b2
cd $R
RAG_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29633 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/b2/bench2.log 2>&1
rc=$?
grep -v "^\[W" gpurun_out/b2/bench2.log | tail -3 | cut -c1-600
exit $rc
