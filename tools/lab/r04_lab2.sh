#!/bin/bash
# tower variants (bench model; H=256 for the base) + GPU tests + bench
set -o pipefail
R=gpurun_out/$1
mkdir -p $R
for v in $2; do
  DCNR_LIB=$PWD/tools/lab_bin/libdcnr_tw_$v.so timeout -k 10 120 python -u tools/tower_probe.py 200 131072 > $R/probe_$v.log 2>&1 || exit 1
done
TOWER_H=256 DCNR_LIB=$PWD/tools/lab_bin/libdcnr_tw_g4.so timeout -k 10 120 python -u tools/tower_probe.py 200 131072 > $R/probe_g4_h256.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $R/gpu_tests.log 2>&1 || exit 1
timeout -k 10 400 python3 -u bench.py > $R/bench.log 2>&1 || exit 1
