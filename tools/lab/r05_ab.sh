#!/bin/bash
# GPU tests of the given files, then a step A/B against lab variants
#   bash tools/lab/r05_ab.sh <tag> "<test files>" "<variants>" [rounds]
set -o pipefail
R=gpurun_out/$1; mkdir -p $R
export TMPDIR=/tmp
if [ -n "$2" ]; then
  timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread $2 > $R/tests.log 2>&1 || exit 1
fi
for v in $3; do bash tools/ab_step.sh $1/ab_$v $v ${4:-2} || exit 1; done
