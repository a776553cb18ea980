#!/bin/bash
# round 6: emb_runs_short_kernel variants (tools/lab_bin/libdcnr_<v>.so): the embedding GPU tests on
# each, then per-kernel times from a kernel trace of a short bench run.
#   bash tools/lab/r06_emb_short.sh <tag> <v1> [v2 ...]
set -o pipefail
R=gpurun_out/$1; shift; mkdir -p $R
export TMPDIR=/tmp
A="--steps 10 --warmup 3 --no-cpu-baseline --no-serving --no-fp32 --no-zipf"
for v in base "$@"; do
  if [ $v = base ]; then unset DCNR_LIB; else export DCNR_LIB=$PWD/tools/lab_bin/libdcnr_$v.so; fi
  if [ $v != base ]; then
    timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_embed_bwd_gpu.py > $R/${v}_tests.log 2>&1 || { echo "$v tests failed"; exit 1; }
  fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$v -o run -- python3 bench.py $A > $R/$v.log 2>&1 || exit 1
  python3 - $R/$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "emb_runs" in r["Name"]:
        print(sys.argv[2], r["Name"][:48], round(float(r["AverageNs"]) / 1000, 1))
PY
done
