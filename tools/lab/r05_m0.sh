#!/bin/bash
# LDS-DMA asm with M0 as a compiler-set input ("{m0}") instead of saved and
# restored inside the statement: GPU suite on the lab build, the tower
# kernel, and the train step
set -o pipefail
R=gpurun_out/r05m0i; mkdir -p $R
ROOT=$(pwd)
DCNR_LIB=$ROOT/tools/lab_bin/libdcnr_m0all.so timeout -k 10 700 python -u -m pytest -x -q --timeout 120 \
  --timeout-method thread -m gpu tests > $R/m0all_tests.log 2>&1 || exit 1
TWOUT=r05m0i/tw VARIANTS="base m0t" bash tools/lab/r05_tw.sh || exit 1
bash tools/ab_bench.sh $R/ab 2 base m0all
