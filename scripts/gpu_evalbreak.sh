set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python benchmarks/eval_breakdown.py > gpurun_out/eb.log 2>&1 && \
timeout -k 10 300 python benchmarks/eval_breakdown.py --wave > gpurun_out/ebw.log 2>&1
