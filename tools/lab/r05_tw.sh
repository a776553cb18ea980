#!/bin/bash
# tower ablations (lab): tower_kernel under rocprofv3 --kernel-trace --stats
# with the production library and lab builds, each twice, interleaved
set -o pipefail
R=gpurun_out/${TWOUT:-r05tw}; mkdir -p $R
ROOT=$(pwd)
export TMPDIR=/tmp
for rep in 1 2; do
  for v in ${VARIANTS:-base nobar nowait nox}; do
    if [ $v = base ]; then L=$ROOT/hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd/lib/libdcnr.so; else L=$ROOT/tools/lab_bin/libdcnr_tw_$v.so; fi
    (cd /tmp && DCNR_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $ROOT/$R/${v}_$rep -o run -- python3 $ROOT/tools/tower_probe.py 131072 > $ROOT/$R/${v}_$rep.log 2>&1) || exit 1
  done
done
