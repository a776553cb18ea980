#!/bin/bash
# scan v4 lab: each tools/lab_bin/libdcnr_<v>.so under rocprofv3 --stats
# (on the GPU box, from the repo root):  bash tools/knn_lab.sh <outdir> v1 v2 ...
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
ROOT=$(pwd)
export TMPDIR=/tmp
for v in "$@"; do
  (cd /tmp && DCNR_LIB=$ROOT/tools/lab_bin/libdcnr_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats \
      --output-format csv -d $ROOT/$OUT/$v -o run -- python3 $ROOT/tools/knn_lab.py > $ROOT/$OUT/$v.log 2>&1) || exit 1
done
