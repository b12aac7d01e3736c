set -o pipefail
timeout -k 10 600 python -m pytest tests/test_gpu_sampling.py tests/test_resnet_gpu.py tests/test_hip_kernels.py tests/test_gpu_cli.py -x -q -m gpu > gpurun_out/t.log 2>&1
