set -o pipefail
mkdir -p gpurun_out
HIP_LAUNCH_BLOCKING=1 AMD_SERIALIZE_KERNEL=3 timeout -k 10 120 python scripts/dbg/ladder_leaves.py > gpurun_out/ladder_leaves.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_ladders.py tests/test_gpu_features.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_ladder.log 2>&1 && \
timeout -k 10 300 python benchmarks/eval_breakdown.py > gpurun_out/eb.log 2>&1 && \
timeout -k 10 120 python benchmarks/mcts_bench.py --lmbda 0 > gpurun_out/mcts_lad.jsonl 2>gpurun_out/mcts_lad.err && \
RAG_LADDERS=gpu timeout -k 10 120 python benchmarks/mcts_bench.py --lmbda 0 >> gpurun_out/mcts_lad.jsonl 2>>gpurun_out/mcts_lad.err
