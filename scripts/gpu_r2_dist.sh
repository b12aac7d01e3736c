set -o pipefail
mkdir -p gpurun_out/dist
timeout -k 10 300 python -u -m pytest tests/test_distributed_search.py tests/test_gpu_search.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dist/tests.log 2>&1 && \
timeout -k 10 200 python benchmarks/mcts_bench.py --moves 2 > gpurun_out/dist/mcts1.log 2>&1 && \
timeout -k 10 200 python benchmarks/mcts_bench.py --distributed --moves 2 > gpurun_out/dist/mcts_dist1.log 2>&1 && \
RAG_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 benchmarks/mcts_bench.py --distributed --moves 2 --threads 8 > gpurun_out/dist/mcts_dist2.log 2>&1 && \
timeout -k 10 200 python benchmarks/converter_bench.py --copies 40 --threads 1,4,16 > gpurun_out/dist/conv.log 2>&1
