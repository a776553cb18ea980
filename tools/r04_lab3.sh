#!/bin/bash
set -o pipefail
R=gpurun_out/$1
mkdir -p $R
for v in $2; do
  DCNR_LIB=$PWD/tools/lab_bin/libdcnr_tw_$v.so timeout -k 10 120 python -u tools/tower_probe.py 200 131072 > $R/probe_$v.log 2>&1 || exit 1
done
for v in $3; do
  DCNR_LIB=$PWD/tools/lab_bin/libdcnr_tw_$v.so timeout -k 10 200 python -u -m pytest tests/test_eval_head_gpu.py -x -q -s --timeout 120 --timeout-method thread > $R/evaltest_$v.log 2>&1 || exit 1
done
bash tools/tower_counters.sh $1
