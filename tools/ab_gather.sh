#!/bin/bash
# gather_probe.py over lab builds: default library first, then each
# tools/lab_bin/libdcnr_<v>.so.   bash tools/ab_gather.sh <tag> "<variants>"
set -o pipefail
R=gpurun_out/$1
mkdir -p $R
timeout -k 10 150 python -u tools/gather_probe.py > $R/gather_base.log 2>&1 || exit 1
for v in $2; do
  DCNR_LIB=$PWD/tools/lab_bin/libdcnr_$v.so timeout -k 10 150 python -u tools/gather_probe.py > $R/gather_$v.log 2>&1 || exit 1
done
timeout -k 10 150 python -u tools/gather_probe.py > $R/gather_base2.log 2>&1 || exit 1
