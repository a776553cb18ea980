#!/bin/bash
# Q=32 top-k lab: the probe with the production library and lab builds
# (bound5 with two 16-query groups per block at 17..32 queries; a 7-bit
# mantissa cut in the minima search), each twice, interleaved
set -o pipefail
R=gpurun_out/r05q32; mkdir -p $R
ROOT=$(pwd)
for rep in 1 2; do
  for v in base qg2 low16 both; do
    if [ $v = base ]; then unset DCNR_LIB; else export DCNR_LIB=$ROOT/tools/lab_bin/libdcnr_$v.so; fi
    timeout -k 10 120 python -u tools/knn_probe.py > $R/${v}_$rep.log 2>&1 || exit 1
  done
done
unset DCNR_LIB
