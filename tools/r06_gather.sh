#!/bin/bash
# round 6: the low-rank train/eval gather front -- probe, then suite/smoke/bench
set -o pipefail
R=gpurun_out/$1; mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/gather_probe.py > $R/gather_probe.log 2>&1 || exit 1
cat $R/gather_probe.log | grep -v amdgpu.ids
bash tools/r06_check.sh $1/check
