#!/bin/bash
# gemm_wsp with the end-of-kernel drain: the flaky embedding-backward
# bit-identity tests 3x, the GPU suite, then a step A/B against gemm_ws
set -o pipefail
R=gpurun_out/$1; mkdir -p $R
export TMPDIR=/tmp
bash tools/lab/r05_flaky.sh $1/flaky base || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $R/tests.log 2>&1 || exit 1
bash tools/ab_step.sh $1/ab nowsp 2 || exit 1
