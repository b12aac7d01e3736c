#!/bin/bash
# PMC counters of the round-3 SL training step kernels and the ResNet step (separate runs,
# counters only, no tracing domains)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc3
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/sl -- python3 $R/bench.py --no-mcts --steps 6 --warmup 2 > $O/sl.log 2>&1 || { tail -5 $O/sl.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/res -- python3 $R/bench.py --model resnet --no-mcts --steps 6 --warmup 2 > $O/res.log 2>&1 || { tail -5 $O/res.log; exit 1; }
cd $R
python tools/pmcsum.py $(find $O/sl -name "*counter_collection.csv" | head -1) > $O/sl_sum.txt 2>&1 || true
python tools/pmcsum.py $(find $O/res -name "*counter_collection.csv" | head -1) > $O/res_sum.txt 2>&1 || true
head -12 $O/sl_sum.txt
head -14 $O/res_sum.txt
