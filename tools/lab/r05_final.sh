#!/bin/bash
# Round-5 final set on one box: GPU suite, smoke, the round profile
# (bench + kernel trace + PMC traffic, tools/profile_round.sh), and the kNN
# PMC passes over tools/knn_lab.py (Q = 1 / 32 / 256).
#   bash tools/lab/r05_final.sh <tag> [part]   part: 1 = tests + smoke + knn PMC, 2 = profile_round
set -o pipefail
R=gpurun_out/$1; mkdir -p $R
export TMPDIR=/tmp
ROOT=$(pwd)
if [ "${2:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests > $R/gpu_tests.log 2>&1 || exit 1
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.log 2>&1 || exit 1
  (cd /tmp && timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $ROOT/$R/knnf -o run \
      -- python3 $ROOT/tools/knn_lab.py > $ROOT/$R/knnf.log 2>&1) || exit 1
  (cd /tmp && timeout -k 10 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $ROOT/$R/knnw -o run \
      -- python3 $ROOT/tools/knn_lab.py > $ROOT/$R/knnw.log 2>&1) || exit 1
  python3 tools/knn_pmc.py $R/knnf/run_counter_collection.csv $R/knnw/run_counter_collection.csv > $R/knn_pmc.txt
else
  bash tools/profile_round.sh $1
fi
