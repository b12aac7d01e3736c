set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof_sl $R/gpurun_out/prof_mcts
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_sl -- python $R/bench.py --steps 20 --warmup 3 --no-mcts > $R/gpurun_out/prof_sl.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_mcts -- python $R/benchmarks/mcts_bench.py --moves 2 > $R/gpurun_out/prof_mcts.log 2>&1 && \
cd $R && timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --model value --no-mcts > gpurun_out/bench_value.log 2>&1 && \
timeout -k 10 300 python bench.py --model resnet --no-mcts > gpurun_out/bench_resnet.log 2>&1
