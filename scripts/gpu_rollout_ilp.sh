set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python scripts/dbg/rollout_ref.py check tests/data/rollout_ref.npz > gpurun_out/rref_check.log 2>&1 ; echo "check rc=$?" >> gpurun_out/rref_check.log
timeout -k 10 200 python -u -m pytest tests/test_gpu_search.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gsearch.log 2>&1 && \
timeout -k 10 200 python benchmarks/rollout_bench.py > gpurun_out/rbench_after.log 2>&1 && \
timeout -k 10 120 python benchmarks/mcts_bench.py --moves 3 > gpurun_out/mcts_after.jsonl 2>gpurun_out/mcts_after.err
