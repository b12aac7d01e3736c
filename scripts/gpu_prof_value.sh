set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof_value
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_value -- python $R/bench.py --model value --no-mcts --steps 20 --warmup 3 > $R/gpurun_out/prof_value.log 2>&1
