set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES --output-format csv -d $R/gpurun_out/pmc/p1 -- python $R/benchmarks/kernel_bench.py > $R/gpurun_out/pmc/p1.log 2>&1 && \
RAG_CONV_PIPE=0 timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES --output-format csv -d $R/gpurun_out/pmc/p0 -- python $R/benchmarks/kernel_bench.py > $R/gpurun_out/pmc/p0.log 2>&1
