#!/bin/bash
# diagnostic: wgrad reduce with OIHW scattered writes vs contiguous writes (wrong layout)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/wreddiag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/a -- python3 $R/scripts/dbg/wgrad_ab.py > $O/a.log 2>&1 &&
RAG_WRED_DIAG=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/b -- python3 $R/scripts/dbg/wgrad_ab.py > $O/b.log 2>&1
rc=$?
for d in a b; do f=$(ls $O/$d/*/*kernel_stats.csv | head -1); grep -i reduce $f | cut -c1-200; done
exit $rc
