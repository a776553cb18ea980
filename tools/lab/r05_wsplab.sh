#!/bin/bash
# which condition makes the gemm_wsp train-step flakiness go away:
# base (wsp), wsplds (wsp alone on its CU: 160 KB LDS), sortmain (the forward's
# id sort on the main stream), nowsp (gemm_ws)
set -o pipefail
bash tools/lab/r05_flaky.sh $1 "base wsplds sortmain nowsp"
