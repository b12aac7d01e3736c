set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/clk
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES --output-format csv -d $R/gpurun_out/clk/p1 -- python3 $R/benchmarks/kernel_bench.py > $R/gpurun_out/clk/p1.log 2>&1 && \
timeout -k 10 120 python3 $R/benchmarks/kernel_bench.py > $R/gpurun_out/clk/kb.log 2>&1 && \
cd $R && timeout -k 10 300 python3 bench.py > gpurun_out/clk/bench.log 2>&1
