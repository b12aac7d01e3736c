set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py tests/test_gpu_models.py tests/test_gpu_search.py tests/test_gpu_cli.py > gpurun_out/vmlp2_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --model value --no-mcts > gpurun_out/bench_value_vmlp.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_vmlp.log 2>&1
