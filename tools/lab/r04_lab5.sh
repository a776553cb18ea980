#!/bin/bash
# Tower lab round: probes of lab variants (default library first), then the
# eval-tower tests with the variants that must stay correct.
#   bash tools/lab/r04_lab5.sh <tag> "<probe variants>" "<test variants>"
set -o pipefail
R=gpurun_out/$1
mkdir -p $R
timeout -k 10 120 python -u tools/tower_probe.py 131072 > $R/probe_base.log 2>&1 || exit 1
for v in $2; do
  DCNR_LIB=$PWD/tools/lab_bin/libdcnr_tw_$v.so timeout -k 10 120 python -u tools/tower_probe.py 131072 > $R/probe_$v.log 2>&1 || exit 1
done
for v in $3; do
  DCNR_LIB=$PWD/tools/lab_bin/libdcnr_tw_$v.so timeout -k 10 200 python -u -m pytest tests/test_eval_head_gpu.py -k "not threshold" -x -q -s --timeout 120 --timeout-method thread > $R/evaltest_$v.log 2>&1 || exit 1
done
