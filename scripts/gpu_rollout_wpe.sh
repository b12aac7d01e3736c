set -o pipefail
mkdir -p gpurun_out
for w in 4 3; do
  RAG_ROLLOUT_WPE=$w timeout -k 10 200 python scripts/dbg/rollout_ref.py check tests/data/rollout_ref.npz > gpurun_out/rref_w$w.log 2>&1 || exit 1
  grep -q "winners equal True lengths equal True logits equal True" gpurun_out/rref_w$w.log || exit 1
done
for w in 4 3 4 3; do
  RAG_ROLLOUT_WPE=$w timeout -k 10 200 python benchmarks/rollout_bench.py >> gpurun_out/rbench_w$w.log 2>&1 || exit 1
done
for w in 4 3; do
  RAG_ROLLOUT_WPE=$w timeout -k 10 120 python benchmarks/mcts_bench.py --moves 3 >> gpurun_out/mcts_w$w.jsonl 2>gpurun_out/mcts_w$w.err || exit 1
done
timeout -k 10 200 python -u -m pytest tests/test_gpu_search.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gsearch.log 2>&1
