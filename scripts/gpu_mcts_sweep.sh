set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/mcts_sweep.jsonl
: > $O
run() { timeout -k 10 120 python benchmarks/mcts_bench.py "$@" >> $O 2>>gpurun_out/sweep.err; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_search.log 2>&1 && \
run --pipeline 2 --rollouts-per-leaf 1 --max-inflight 4 && \
run --pipeline 2 --rollouts-per-leaf 1 --max-inflight 8 && \
run --pipeline 2 --rollouts-per-leaf 1 --max-inflight 8 --batch 512 && \
run --pipeline 2 --rollouts-per-leaf 4 --max-inflight 8 && \
run --pipeline 2 --rollouts-per-leaf 1 --max-inflight 8 --moves 4 --playouts 16384
