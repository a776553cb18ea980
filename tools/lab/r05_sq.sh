#!/bin/bash
# SQ counters of tools/bench_gemm.py for the default library and lab variants
#   bash tools/lab/r05_sq.sh <tag> "<variants>"
set -o pipefail
T=$1
SQ_PROG="tools/bench_gemm.py" bash tools/sq_counters.sh $T/base || exit 1
for v in $2; do
  DCNR_LIB=$PWD/tools/lab_bin/libdcnr_$v.so SQ_PROG="tools/bench_gemm.py" bash tools/sq_counters.sh $T/$v || exit 1
done
