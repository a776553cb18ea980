#!/bin/bash
# LDS-DMA through the compiler intrinsic (dma16b) instead of the M0-saving
# asm: correctness of the lab builds, the tower kernel, and the train step
set -o pipefail
R=gpurun_out/r05dmab; mkdir -p $R
ROOT=$(pwd)
DCNR_LIB=$ROOT/tools/lab_bin/libdcnr_tw_bl.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread tests/test_eval_head_gpu.py > $R/bl_tests.log 2>&1 || exit 1
DCNR_LIB=$ROOT/tools/lab_bin/libdcnr_wsdw.so timeout -k 10 700 python -u -m pytest -x -q --timeout 120 \
  --timeout-method thread -m gpu tests > $R/wsdw_tests.log 2>&1 || exit 1
TWOUT=r05dmab/tw VARIANTS="base bl" bash tools/lab/r05_tw.sh || exit 1
bash tools/ab_bench.sh $R/ab 2 base ws dw wsdw
