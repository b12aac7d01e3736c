set -o pipefail
timeout -k 10 600 python -m pytest tests/test_gpu_search.py -x -q -m gpu > gpurun_out/t.log 2>&1 && \
timeout -k 10 300 python benchmarks/mcts_bench.py --playouts 4096 > gpurun_out/mcts.log 2>&1 && \
timeout -k 10 300 python benchmarks/mcts_bench.py --playouts 4096 --rollouts-per-leaf 16 --batch 512 >> gpurun_out/mcts.log 2>&1 && \
timeout -k 10 300 python benchmarks/mcts_bench.py --playouts 2048 --lmbda 0 >> gpurun_out/mcts.log 2>&1
