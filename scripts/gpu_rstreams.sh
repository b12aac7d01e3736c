set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/rstreams.jsonl
: > $OUT
for ns in 4 3 2 6; do
  echo "streams=$ns" >> $OUT
  RAG_ROLLOUT_STREAMS=$ns timeout -k 10 120 python benchmarks/mcts_bench.py >> $OUT 2>gpurun_out/rs.err || exit 1
done
echo "streams=4 inflight=8" >> $OUT
timeout -k 10 120 python benchmarks/mcts_bench.py --max-inflight 8 >> $OUT 2>>gpurun_out/rs.err || exit 1
echo "streams=6 inflight=8" >> $OUT
RAG_ROLLOUT_STREAMS=6 timeout -k 10 120 python benchmarks/mcts_bench.py --max-inflight 8 >> $OUT 2>>gpurun_out/rs.err || exit 1
echo "streams=4 prio=1" >> $OUT
RAG_ROLLOUT_PRIORITY=1 timeout -k 10 120 python benchmarks/mcts_bench.py >> $OUT 2>>gpurun_out/rs.err || exit 1
echo "streams=3 batch512" >> $OUT
RAG_ROLLOUT_STREAMS=3 timeout -k 10 120 python benchmarks/mcts_bench.py --batch 512 >> $OUT 2>>gpurun_out/rs.err || exit 1
