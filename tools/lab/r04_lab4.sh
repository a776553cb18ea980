#!/bin/bash
# GPU tests, tower probes (default library + lab variants), bench line.
#   bash tools/lab/r04_lab4.sh <tag> "<lab variants>"
set -o pipefail
R=gpurun_out/$1
mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $R/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/tower_probe.py 131072 > $R/probe_base.log 2>&1 || exit 1
for v in $2; do
  DCNR_LIB=$PWD/tools/lab_bin/libdcnr_tw_$v.so timeout -k 10 120 python -u tools/tower_probe.py 131072 > $R/probe_$v.log 2>&1 || exit 1
done
timeout -k 10 120 python -u tools/tower_probe.py 4096 8192 16384 32768 > $R/probe_small.log 2>&1 || exit 1
timeout -k 10 400 python3 -u bench.py > $R/bench.log 2>&1 || exit 1
