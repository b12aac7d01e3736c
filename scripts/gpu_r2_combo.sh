#!/bin/bash
# SL quick check (kernel tests, bench, step trace) then the MCTS bound sweep
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 700 bash scripts/gpu_r2_slq.sh head && timeout -k 10 600 bash scripts/gpu_r2_mctsx.sh
