#!/bin/bash
# One GPU round-trip (from the repo root on the box): GPU tests, then the
# default bench line.   bash tools/lab/r04_check.sh <tag> [pytest -k expr]
set -o pipefail
R=gpurun_out/${1:-r04x}
mkdir -p $R
export TMPDIR=/tmp
K=${2:+-k "$2"}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread $K > $R/gpu_tests.log 2>&1 || exit 1
timeout -k 10 400 python3 -u bench.py > $R/bench.log 2>&1 || exit 1
