set -o pipefail
mkdir -p gpurun_out/pass
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pass/gpu_tests.log 2>&1 && \
timeout -k 10 200 python benchmarks/converter_bench.py --copies 40 --threads 1,4,16 > gpurun_out/pass/conv.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/pass/bench.log 2>&1
