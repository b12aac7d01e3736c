set -o pipefail
timeout -k 10 400 python -m pytest tests/test_hip_kernels.py -x -q -m gpu > gpurun_out/t.log 2>&1
