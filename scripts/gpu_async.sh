set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/async.jsonl
: > $OUT
for cfg in "0 2" "1 2" "1 3" "1 4"; do
  set -- $cfg
  echo "async=$1 pipeline=$2" >> $OUT
  RAG_ASYNC_EVAL=$1 timeout -k 10 120 python benchmarks/mcts_bench.py --moves 3 --pipeline $2 >> $OUT 2>gpurun_out/as.err || exit 1
done
echo "async=1 pipeline=3 lmbda0" >> $OUT
timeout -k 10 120 python benchmarks/mcts_bench.py --moves 3 --pipeline 3 --lmbda 0 >> $OUT 2>>gpurun_out/as.err || exit 1
echo "async=1 pipeline=3 batch512" >> $OUT
timeout -k 10 120 python benchmarks/mcts_bench.py --moves 3 --pipeline 3 --batch 512 >> $OUT 2>>gpurun_out/as.err || exit 1
