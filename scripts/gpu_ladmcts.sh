set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/ladmcts.jsonl
: > $OUT
for cfg in "host 0 2" "gpu 0 2" "gpu 1 2" "gpu 1 3" "gpu 0 3"; do
  set -- $cfg
  echo "ladders=$1 async=$2 pipeline=$3" >> $OUT
  RAG_LADDERS=$1 RAG_ASYNC_EVAL=$2 timeout -k 10 120 python benchmarks/mcts_bench.py --moves 3 --pipeline $3 >> $OUT 2>gpurun_out/lm.err || exit 1
done
echo "ladders=gpu async=1 pipeline=2 lmbda0" >> $OUT
RAG_LADDERS=gpu timeout -k 10 120 python benchmarks/mcts_bench.py --moves 3 --lmbda 0 >> $OUT 2>>gpurun_out/lm.err || exit 1
