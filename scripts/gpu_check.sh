set -o pipefail
timeout -k 10 400 python -m pytest tests/test_gpu_search.py tests/test_gpu_features.py -x -q -m gpu > gpurun_out/t.log 2>&1 && \
timeout -k 10 300 python benchmarks/mcts_bench.py --playouts 4096 > gpurun_out/mcts.log 2>&1 && \
timeout -k 10 300 python benchmarks/mcts_bench.py --playouts 8192 --batch 512 >> gpurun_out/mcts.log 2>&1 && \
timeout -k 10 300 python benchmarks/mcts_bench.py --playouts 8192 --batch 256 --rollouts-per-leaf 2 >> gpurun_out/mcts.log 2>&1 && \
timeout -k 10 300 python benchmarks/mcts_bench.py --playouts 4096 --lmbda 0 >> gpurun_out/mcts.log 2>&1
