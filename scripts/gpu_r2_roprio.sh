#!/bin/bash
# rollout stream priority vs the network (default) stream: low (1) / default (0) / high (-1)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/roprio
mkdir -p $O
cd $R
python -c "import torch; print('priority_range', torch.cuda.Stream.priority_range())"
run() { n=$1; p=$2; RAG_ROLLOUT_PRIORITY=$p timeout -k 10 150 python -u benchmarks/mcts_bench.py --moves 6 > $O/$n.log 2>&1 || exit 1; echo $n $(tail -1 $O/$n.log | cut -c1-60); }
for rep in 1 2; do run p0_$rep 0; run p1_$rep 1; run pm1_$rep -1; done
