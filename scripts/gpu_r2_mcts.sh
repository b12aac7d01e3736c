set -o pipefail
mkdir -p gpurun_out/r2m
timeout -k 10 120 python scripts/dbg/host_scaling.py > gpurun_out/r2m/host_scaling.log 2>&1 && \
timeout -k 10 300 python benchmarks/mcts_bench.py --moves 2 > gpurun_out/r2m/mcts_bench.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_ladders.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2m/tests.log 2>&1
