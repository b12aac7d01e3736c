set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_hip.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_models.log 2>&1 && \
RAG_WGRAD_SLAB=0 timeout -k 10 180 python benchmarks/kernel_bench.py > gpurun_out/kb_nows.log 2>&1 && \
timeout -k 10 180 python benchmarks/kernel_bench.py > gpurun_out/kb_ws.log 2>&1 && \
RAG_WGRAD_SLAB=0 timeout -k 10 300 python bench.py --no-mcts > gpurun_out/bench_nows.log 2>&1 && \
timeout -k 10 300 python bench.py --no-mcts > gpurun_out/bench_ws.log 2>&1
