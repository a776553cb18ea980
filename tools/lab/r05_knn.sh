#!/bin/bash
# kNN round-5 check: the kNN GPU tests, the probe's per-call times, and a
# rocprofv3 kernel trace of the probe split per call.
#   bash tools/lab/r05_knn.sh <tag> [variant-lib-name]
set -o pipefail
R=gpurun_out/$1; mkdir -p $R
export TMPDIR=/tmp
ROOT=$(pwd)
[ -n "$2" ] && export DCNR_LIB=$ROOT/tools/lab_bin/libdcnr_$2.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_knn_sharded_gpu.py tests/test_parity_gpu.py -k "knn or cosine or topk or similar" > $R/tests.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/knn_probe.py > $R/probe.log 2>&1 || exit 1
(cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$R/prof -o run \
  -- python3 $ROOT/tools/knn_probe.py > $ROOT/$R/prof.log 2>&1) || exit 1
f=$(find $R/prof -name '*kernel_trace.csv' | head -1)
python3 tools/knn_trace.py $f 13 > $R/trace.txt 2>&1
