#!/bin/bash
# round 6: the batched exact fallback (Q > 16) -- knn tests, the all-overflow probe,
# and the kNN probe A/B against the previous knn.hip (tools/lab_bin/libdcnr_knnold.so)
set -o pipefail
R=gpurun_out/$1; mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity_gpu.py tests/test_knn_sharded_gpu.py \
  -k "knn" > $R/knn_tests.log 2>&1; rc=$?
tail -n 2 $R/knn_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/knn_overflow_probe.py > $R/overflow.log 2>&1 || exit 1
grep -v amdgpu.ids $R/overflow.log
for v in new old new2 old2; do
  if [ ${v%2} = old ]; then export DCNR_LIB=$PWD/tools/lab_bin/libdcnr_knnold.so; else unset DCNR_LIB; fi
  timeout -k 10 300 python -u tools/knn_probe.py > $R/knn_probe_$v.log 2>&1 || exit 1
  echo "== $v"; grep "^Q=" $R/knn_probe_$v.log
done
