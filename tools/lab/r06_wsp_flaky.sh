#!/bin/bash
# round 6: which change to gemm_wsp's last tiles removes the train-step
# run-to-run differences (tests/test_embed_bwd_gpu.py's bit-identity pair)
#   bash tools/lab/r06_wsp_flaky.sh <tag> "<variants>"   (libs from r06_wsp_build.sh)
set -o pipefail
bash tools/lab/r05_flaky.sh $1 "$2"
cat gpurun_out/$1/summary.txt
