set -o pipefail
timeout -k 10 400 python -m pytest tests/test_hip_kernels.py tests/test_gpu_models.py -x -q -m gpu > gpurun_out/t.log 2>&1 && \
timeout -k 10 200 python benchmarks/kernel_bench.py > gpurun_out/kb.log 2>&1 && \
RAG_CONV_PIPE=0 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-mcts > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-mcts >> gpurun_out/bench.log 2>&1
