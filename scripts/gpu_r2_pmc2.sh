#!/bin/bash
# PMC counters of the round-2 SL training step kernels (separate run, kernel trace only)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc -- python3 $R/bench.py --no-mcts --steps 6 --warmup 2 > $O/pmc.log 2>&1
rc=$?
ls -R $O/pmc | head -5
exit $rc
