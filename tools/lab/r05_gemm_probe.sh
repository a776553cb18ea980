#!/bin/bash
# bench_gemm.py for the default library and lab variants: bash tools/lab/r05_gemm_probe.sh <tag> "<variants>"
set -o pipefail
R=gpurun_out/$1; mkdir -p $R
timeout -k 10 120 python -u tools/bench_gemm.py > $R/gemm_base.log 2>&1 || exit 1
for v in $2; do
  DCNR_LIB=$PWD/tools/lab_bin/libdcnr_$v.so timeout -k 10 120 python -u tools/bench_gemm.py > $R/gemm_$v.log 2>&1 || exit 1
done
timeout -k 10 120 python -u tools/bench_gemm.py > $R/gemm_base2.log 2>&1 || exit 1
grep -H "K=512 N=512" $R/gemm_*.log > $R/summary.txt
