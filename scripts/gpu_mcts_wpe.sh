set -o pipefail
mkdir -p gpurun_out
for w in 4 3 4 3 4 3; do
  RAG_ROLLOUT_WPE=$w timeout -k 10 120 python benchmarks/mcts_bench.py --moves 4 >> gpurun_out/mcts2_w$w.jsonl 2>>gpurun_out/mcts2_w$w.err || exit 1
done
