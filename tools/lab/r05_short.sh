#!/bin/bash
# grouped short-run embedding sums: bit-exact tests, then a step A/B against the one-thread-per-run kernel
set -o pipefail
R=gpurun_out/$1; mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_embed_bwd_gpu.py \
  tests/test_row_map_gpu.py tests/test_stages_gpu.py tests/test_dp_gpu.py > $R/tests.log 2>&1 || exit 1
bash tools/ab_step.sh $1/ab oldshort 2 || exit 1
