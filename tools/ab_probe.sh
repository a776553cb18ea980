#!/bin/bash
# A/B of lab builds with one probe script: default library, then each
# tools/lab_bin/libdcnr_<v>.so, then the default again (box drift check).
#   bash tools/ab_probe.sh <tag> <probe.py> "<variants>" [probe args]
set -o pipefail
R=gpurun_out/$1; P=$2; V=$3; shift 3
mkdir -p $R
n=$(basename $P .py)
timeout -k 10 150 python -u $P "$@" > $R/${n}_base.log 2>&1 || exit 1
for v in $V; do
  DCNR_LIB=$PWD/tools/lab_bin/libdcnr_$v.so timeout -k 10 150 python -u $P "$@" > $R/${n}_$v.log 2>&1 || exit 1
done
timeout -k 10 150 python -u $P "$@" > $R/${n}_base2.log 2>&1 || exit 1
