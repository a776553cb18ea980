#!/bin/bash
# One GPU round-trip (from the repo root on the box): GPU tests, the kNN probe
# under rocprofv3 --stats, the gemm_ws lab clock passes, the default bench.
#   bash tools/lab/r03_check.sh <tag>
set -o pipefail
R=gpurun_out/${1:-r03x}
mkdir -p $R
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $R/gpu_tests.log 2>&1 || exit 1
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$R/knnprof -o run -- \
    python3 $ROOT/tools/knn_probe.py > $ROOT/$R/knn_probe.log 2>&1) || exit 1
timeout -k 10 400 python3 bench.py > $R/bench.log 2>&1 || exit 1
