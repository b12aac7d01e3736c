set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof_mcts_vmlp
cd $R && timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py tests/test_gpu_models.py tests/test_gpu_search.py > gpurun_out/vmlp_tests.log 2>&1 && \
timeout -k 10 300 python benchmarks/mcts_bench.py --moves 4 > gpurun_out/mcts_bench_vmlp.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_mcts_vmlp -- python $R/benchmarks/mcts_bench.py --moves 2 > $R/gpurun_out/prof_mcts_vmlp.log 2>&1
