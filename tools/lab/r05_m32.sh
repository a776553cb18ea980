#!/bin/bash
# 32x32x16 tower (lab build): the eval-tower tests against it, then the
# kernel timing beside the production library
set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
DCNR_LIB=$ROOT/tools/lab_bin/libdcnr_tw_m32ns.so timeout -k 10 400 python -u -m pytest -x -v --timeout 300 \
  --timeout-method thread tests/test_eval_head_gpu.py > gpurun_out/r05m32_tests.log 2>&1 || exit 1
TWOUT=r05m32 VARIANTS="${VARIANTS:-base m32 m32ns m32a5}" bash tools/lab/r05_tw.sh
