#!/bin/bash
# round 6: the BN-backward row pass folded into the dX GEMMs -- the train-path GPU tests,
# then a step A/B against the previous library (tools/lab_bin/libdcnr_old.so)
set -o pipefail
R=gpurun_out/$1; mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > $R/gpu_tests.log 2>&1; rc=$?
tail -n 3 $R/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab_step.sh $1/ab old 3 || exit 1
cat $R/ab/summary.txt
