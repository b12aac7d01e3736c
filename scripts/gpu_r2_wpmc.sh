set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/wp
cd /tmp && export TMPDIR=/tmp
timeout -k 10 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/wp/pmc -- python3 $R/benchmarks/kernel_bench.py > $R/gpurun_out/wp/pmc.log 2>&1 && \
cd $R && timeout -k 10 300 python bench.py > gpurun_out/wp/bench.log 2>&1
