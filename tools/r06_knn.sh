#!/bin/bash
# round 6: the split exact fallback of scan v4 -- knn tests, the all-overflow probe, the kNN leg's probe
set -o pipefail
R=gpurun_out/$1; mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity_gpu.py tests/test_knn_sharded_gpu.py \
  -k "knn" > $R/knn_tests.log 2>&1; rc=$?
tail -n 2 $R/knn_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/knn_overflow_probe.py > $R/overflow.log 2>&1 || exit 1
grep -v amdgpu.ids $R/overflow.log
timeout -k 10 300 python -u tools/knn_probe.py > $R/knn_probe.log 2>&1 || exit 1
grep -v amdgpu.ids $R/knn_probe.log
