set -o pipefail
export PYTHONUNBUFFERED=1 PYTHONPATH=.
mkdir -p gpurun_out
for t in 16; do for b in 0 1; do timeout -k 10 120 python scripts/dbg/select_ab.py $t $b >> gpurun_out/g3_ab.log 2>&1 || exit 1; done; done
for t in 8 16; do timeout -k 10 120 python benchmarks/mcts_null_bench.py --distributed --mode master --threads $t --playouts 65536 >> gpurun_out/g3_null.log 2>&1 || exit 2; done
