#!/bin/bash
# round 6: gemm_wsp shipped with the store fix -- the step's stored tensors
# compared whole over 16 repeats, the embedding bit-identity pair 3x, then the
# GPU suite, smoke and bench (tools/r06_check.sh)
set -o pipefail
R=gpurun_out/$1; mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/lab/debug_wsp2.py 16 > $R/debug_wsp2.log 2>&1 || exit 1
tail -n 1 $R/debug_wsp2.log
bash tools/lab/r05_flaky.sh $1/flaky base || exit 1
cat $R/flaky/summary.txt
bash tools/r06_check.sh $1/check
