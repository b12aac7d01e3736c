set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES --output-format csv -d $R/gpurun_out/pmc2/p1 -- python $R/benchmarks/kernel_bench.py > $R/gpurun_out/pmc2/p1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_INSTS_BRANCH SQ_WAVES --output-format csv -d $R/gpurun_out/pmc2/p2 -- python $R/benchmarks/kernel_bench.py > $R/gpurun_out/pmc2/p2.log 2>&1
