#!/bin/bash
# gemm_ws epilogue ping-pong: bit-identity tests, the GEMM probe, step A/B
set -o pipefail
R=gpurun_out/$1; mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stages_gpu.py \
  tests/test_embed_bwd_gpu.py tests/test_row_map_gpu.py > $R/tests.log 2>&1 || exit 1
bash tools/lab/r05_flaky.sh $1/flaky base || exit 1
bash tools/lab/r05_gemm_probe.sh $1/probe "ppodd nopp" || exit 1
bash tools/ab_step.sh $1/ab_nopp nopp 2 || exit 1
bash tools/ab_step.sh $1/ab_ppodd ppodd 1 || exit 1
