#!/bin/bash
# round 6: where gemm_wsp's train-step differences land, per lab variant
# (rows / tile rows / column waves of the differing h0 elements)
#   bash tools/lab/r06_wsp_rows.sh <tag> "<variants>"   (libs from r06_wsp_build.sh)
set -o pipefail
R=gpurun_out/$1; mkdir -p $R
for v in $2; do
  DCNR_LIB=$PWD/tools/lab_bin/libdcnr_$v.so timeout -k 10 150 python -u tools/lab/debug_wsp2.py 8 > $R/$v.log 2>&1 || exit 1
done
grep -h "rep\|rows\|DIFFERS\|ALL SAME" $R/*.log | cut -c1-300
