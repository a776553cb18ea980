#!/bin/bash
# round 6: one train step's kernel timeline for the default library and a lab build
#   bash tools/lab/r06_timeline_ab.sh <tag> <variant>
set -o pipefail
export TMPDIR=/tmp
R=gpurun_out/$1; mkdir -p $R
A="--steps 20 --warmup 5 --no-cpu-baseline --no-serving --no-fp32 --no-zipf"
for v in base $2; do
  if [ $v = base ]; then unset DCNR_LIB; else export DCNR_LIB=$PWD/tools/lab_bin/libdcnr_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$v -o run -- python3 bench.py $A > $R/$v.log 2>&1 || exit 1
  python3 tools/step_timeline.py $R/$v/run_kernel_trace.csv --step 12 --all > $R/timeline_$v.txt || exit 1
  head -1 $R/timeline_$v.txt; grep -A20 "main-queue gaps" $R/timeline_$v.txt
done
