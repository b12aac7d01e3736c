set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/rgroup.jsonl
: > $OUT
for cfg in "4 1" "4 2" "4 3" "4 4" "6 1" "6 2" "6 3" "6 4"; do
  set -- $cfg
  echo "streams=$1 group=$2" >> $OUT
  RAG_ROLLOUT_STREAMS=$1 timeout -k 10 120 python benchmarks/mcts_bench.py --moves 3 --rollout-group $2 >> $OUT 2>gpurun_out/rg.err || exit 1
done
echo "streams=4 group=2 batch512" >> $OUT
RAG_ROLLOUT_STREAMS=4 timeout -k 10 120 python benchmarks/mcts_bench.py --moves 3 --rollout-group 2 --batch 512 >> $OUT 2>>gpurun_out/rg.err || exit 1
