#!/bin/bash
# rollout kernel change: bit-exact tests, standalone throughput, instruction counts
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ro
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  $R/tests/test_gpu_search.py -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
timeout -k 10 120 python -u $R/benchmarks/rollout_bench.py > $O/rollout.jsonl 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH --output-format csv -d $O/p1 -- python3 $R/scripts/dbg/rollout_one.py 4096 > $O/p1.log 2>&1
rc=$?
tail -1 $O/tests.log; grep games $O/rollout.jsonl; grep games $O/p1.log
exit $rc
