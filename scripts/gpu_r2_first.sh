set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r2a
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2a/gpu_tests.log 2>&1 && \
timeout -k 10 200 python bench.py > gpurun_out/r2a/bench.log 2>&1 && \
bash scripts/gpu_r2_clock.sh
