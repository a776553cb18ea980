#!/bin/bash
# round 6: low-rank gather front -- wave count and x0 store policy (probe A/B, then step A/B)
set -o pipefail
bash tools/ab_probe.sh $1 tools/gather_probe.py "$2" || exit 1
grep -h "gather_cross" gpurun_out/$1/gather_probe_*.log
for v in $3; do bash tools/ab_step.sh $1/ab_$v $v 2 || exit 1; cat gpurun_out/$1/ab_$v/summary.txt; done
