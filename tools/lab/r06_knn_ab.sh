#!/bin/bash
# round 6: kNN probe A/B -- default library and lab builds (tools/lab_bin/libdcnr_<v>.so), twice
set -o pipefail
R=gpurun_out/$1; mkdir -p $R
for r in 1 2; do
  for v in base $2; do
    if [ $v = base ]; then unset DCNR_LIB; else export DCNR_LIB=$PWD/tools/lab_bin/libdcnr_$v.so; fi
    timeout -k 10 300 python -u tools/knn_probe.py > $R/${v}_$r.log 2>&1 || exit 1
    echo "$v $r $(grep -E '^Q=(1|32|256):' $R/${v}_$r.log | awk '{print $2}' | tr '\n' ' ')"
  done
done
