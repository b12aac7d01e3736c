set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof_mcts_final
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_mcts_final -- python $R/benchmarks/mcts_bench.py --moves 2 > $R/gpurun_out/prof_mcts_final.log 2>&1 && \
cd $R && timeout -k 10 300 python benchmarks/mcts_bench.py --moves 4 > gpurun_out/mcts_bench_final.log 2>&1 && \
timeout -k 10 300 python benchmarks/rollout_bench.py > gpurun_out/rollout_bench_final.log 2>&1
