#!/bin/bash
set -o pipefail
R=gpurun_out/$1
mkdir -p $R
for v in $2; do
  DCNR_LIB=$PWD/tools/lab_bin/libdcnr_tw_$v.so timeout -k 10 120 python -u tools/tower_probe.py 200 131072 > $R/probe_$v.log 2>&1 || exit 1
done
for v in $3; do
  DCNR_LIB=$PWD/tools/lab_bin/libdcnr_tw_$v.so timeout -k 10 200 python -u -m pytest tests/test_eval_head_gpu.py -k "not threshold" -x -q -s --timeout 120 --timeout-method thread > $R/evaltest_$v.log 2>&1 || exit 1
done
bash tools/tower_counters.sh $1
[ -n "$4" ] || exit 0
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -k cosine -x -v --timeout 150 --timeout-method thread > $R/knn_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/knn_probe.py > $R/knn_probe.log 2>&1
DCNR_LIB=$PWD/tools/lab_bin/libdcnr_knn_km.so timeout -k 10 120 python -u tools/knn_probe.py > $R/knn_probe_km.log 2>&1
