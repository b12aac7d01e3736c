set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/wab
cd $R
timeout -k 10 120 python scripts/dbg/wgrad_ab.py > gpurun_out/wab/ab.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py tests/test_gpu_models.py tests/test_resnet_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wab/tests.log 2>&1 && \
timeout -k 10 200 python bench.py --no-mcts > gpurun_out/wab/bench.log 2>&1
