#!/bin/bash
# round 5: the pipelined forward GEMM (gemm_wsp.hip) -- parity, kernel A/B, step A/B
#   bash tools/lab/r05_wsp.sh <tag> "<kernel variants>" "<step variants>"
set -o pipefail
R=gpurun_out/$1; mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_parity_gpu.py -k "linear or f3 or bf16 or fused_trainer" tests/test_stages_gpu.py \
  tests/test_bf16_train_gpu.py > $R/tests.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/bench_gemm.py > $R/gemm_base.log 2>&1 || exit 1
for v in $2; do
  DCNR_LIB=$PWD/tools/lab_bin/libdcnr_$v.so timeout -k 10 120 python -u tools/bench_gemm.py > $R/gemm_$v.log 2>&1 || exit 1
done
for v in $3; do bash tools/ab_step.sh $1/ab_$v $v 2 || exit 1; done
