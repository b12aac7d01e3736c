set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_distributed_search.py tests/test_gpu_search.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/g1_tests.log 2>&1 || exit 1
for t in 8 16; do timeout -k 10 120 python benchmarks/mcts_null_bench.py --distributed --mode master --threads $t --playouts 65536 >> gpurun_out/g1_null.log 2>&1 || exit 2; done
for n in 2 4 8; do timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500+n)) benchmarks/mcts_null_bench.py --distributed --mode master --threads 2 --threads-master 8 --playouts 65536 >> gpurun_out/g1_null.log 2>&1 || exit 3; done
timeout -k 10 200 python benchmarks/mcts_bench.py --distributed --moves 3 > gpurun_out/g1_mcts_dist1.log 2>&1 || exit 4
timeout -k 10 200 python benchmarks/mcts_bench.py --moves 3 > gpurun_out/g1_mcts_single.log 2>&1 || exit 5
