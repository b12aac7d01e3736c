#!/bin/bash
# rehearse the driver's N>1 bench path with 2 ranks on one GPU (gloo; the driver uses RCCL on 8
# GPUs): SL policy (headline, with the shared-root MCTS phase), value net, ResNet (BN fusion + DP)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/dp2
mkdir -p $O
cd $R
RAG_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 2 --steps 10 --warmup 3 > $O/sl.log 2>&1 || { tail -30 $O/sl.log; exit 1; }
grep "^{" $O/sl.log | cut -c1-300
RAG_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29632 bench.py --gpus 2 --steps 10 --warmup 3 --model resnet --no-mcts > $O/res.log 2>&1 || { tail -30 $O/res.log; exit 1; }
grep "^{" $O/res.log | cut -c1-300
