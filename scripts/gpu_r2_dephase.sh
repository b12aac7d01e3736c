#!/bin/bash
# experiment: delay the second-round conv_tap blocks so the two blocks of a CU run out of phase
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/dephase
mkdir -p $O
cd $R
for d in 0 1 2 3 0; do
RAG_CONV_DEPHASE=$d VARIANTS=2 B=256 timeout -k 10 120 python -u scripts/dbg/conv_ab.py > $O/ab_$d.json 2> $O/ab_$d.err || { tail -5 $O/ab_$d.err; exit 1; }
echo $d $(cat $O/ab_$d.json)
done
