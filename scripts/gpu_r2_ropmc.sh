#!/bin/bash
# rollout kernel instruction mix (PMC, one pass per counter group)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ropmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH --output-format csv -d $O/p1 -- python3 $R/scripts/dbg/rollout_one.py 4096 > $O/p1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY --output-format csv -d $O/p2 -- python3 $R/scripts/dbg/rollout_one.py 4096 > $O/p2.log 2>&1
rc=$?
tail -2 $O/p1.log
exit $rc
