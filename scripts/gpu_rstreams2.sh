set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/rstreams2.jsonl
: > $OUT
for cfg in "4 4" "6 8" "8 8" "8 12" "12 12" "12 16" "16 16" "16 24"; do
  set -- $cfg
  echo "streams=$1 inflight=$2" >> $OUT
  RAG_ROLLOUT_STREAMS=$1 timeout -k 10 120 python benchmarks/mcts_bench.py --moves 3 --max-inflight $2 >> $OUT 2>gpurun_out/rs.err || exit 1
done
echo "streams=12 inflight=16 batch512" >> $OUT
RAG_ROLLOUT_STREAMS=12 timeout -k 10 120 python benchmarks/mcts_bench.py --moves 3 --max-inflight 16 --batch 512 >> $OUT 2>>gpurun_out/rs.err || exit 1
