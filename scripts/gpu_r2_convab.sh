set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/cab2
cd $R
VARIANTS=2,8,9 timeout -k 10 120 python scripts/dbg/conv_ab.py > gpurun_out/cab2/ab.log 2>&1

