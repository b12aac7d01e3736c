#!/bin/bash
# block-scaled fp16 wgrad partials: kernel tests (-s: prints the partial error), DP check, A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/fp16
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py tests/test_gpu_models.py -x -q -s --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
RAG_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29631 scripts/dbg/dp_replica_check.py > $O/dp2.log 2>&1 || { tail -20 $O/dp2.log; exit 1; }
for rep in 1 2; do
RAG_WGRAD_PART=fp32 timeout -k 10 200 python -u bench.py --no-mcts --steps 60 > $O/p32_$rep.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --no-mcts --steps 60 > $O/p16_$rep.log 2>&1 || exit 1
done
grep "rel err" $O/tests.log; tail -1 $O/tests.log; grep -E '^\{' $O/dp2.log
for f in $O/p*.log; do echo $(basename $f) $(tail -1 $f | grep -o '"value": [0-9.]*'); done
