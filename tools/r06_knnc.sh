#!/bin/bash
# round 6: batched exact fallback -- knn tests, then the all-overflow probe for the
# default library and lab builds (tools/lab_bin/libdcnr_<v>.so), and the kNN probe
set -o pipefail
R=gpurun_out/$1; mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity_gpu.py tests/test_knn_sharded_gpu.py \
  -k "knn" > $R/knn_tests.log 2>&1; rc=$?
tail -n 2 $R/knn_tests.log
[ $rc -eq 0 ] || exit $rc
for v in base $2; do
  if [ $v = base ]; then unset DCNR_LIB; else export DCNR_LIB=$PWD/tools/lab_bin/libdcnr_$v.so; fi
  timeout -k 10 300 python -u tools/knn_overflow_probe.py > $R/overflow_$v.log 2>&1 || exit 1
  echo "== $v"; grep "all-overflow\|Q= 256 clean" $R/overflow_$v.log
done
unset DCNR_LIB
timeout -k 10 300 python -u tools/knn_probe.py > $R/knn_probe.log 2>&1 || exit 1
grep "^Q=" $R/knn_probe.log
