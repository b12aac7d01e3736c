#!/bin/bash
# SL / value / resnet throughput sweep on one MI355X (each step time-limited; stops at first failure).
set -o pipefail
mkdir -p gpurun_out/sweep
O=gpurun_out/sweep/results.jsonl
: > $O
for b in 128 256 512 1024; do
  timeout -k 10 180 python bench.py --no-mcts --batch $b --steps 30 --warmup 5 > gpurun_out/sweep/policy_b$b.log 2>&1 || exit 1
  tail -1 gpurun_out/sweep/policy_b$b.log >> $O
done
timeout -k 10 180 python bench.py --no-mcts --model value --steps 30 --warmup 5 > gpurun_out/sweep/value.log 2>&1 || exit 1
tail -1 gpurun_out/sweep/value.log >> $O
timeout -k 10 180 python bench.py --no-mcts --model resnet --steps 30 --warmup 5 > gpurun_out/sweep/resnet.log 2>&1 || exit 1
tail -1 gpurun_out/sweep/resnet.log >> $O
