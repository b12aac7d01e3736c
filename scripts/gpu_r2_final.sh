#!/bin/bash
# final round-2 check: full GPU suite, smoke, benches, then the 2-rank gloo bench rehearsal
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 bash scripts/gpu_r2_end.sh && timeout -k 10 700 bash scripts/gpu_r2_dp2.sh
