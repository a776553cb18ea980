#!/bin/bash
# Train-step A/B: the default library and tools/lab_bin/libdcnr_<v>.so
# alternating, each a short bench run (no CPU baseline, serving, fp32 or
# Zipf legs).   bash tools/ab_step.sh <tag> <variant> [rounds]
set -o pipefail
R=gpurun_out/$1; V=$2; N=${3:-2}
mkdir -p $R
A="--steps 20 --warmup 5 --no-cpu-baseline --no-serving --no-fp32 --no-zipf"
for i in $(seq $N); do
  timeout -k 10 300 python3 -u bench.py $A > $R/base_$i.log 2>&1 || exit 1
  DCNR_LIB=$PWD/tools/lab_bin/libdcnr_$V.so timeout -k 10 300 python3 -u bench.py $A > $R/${V}_$i.log 2>&1 || exit 1
done
for f in $R/*_[0-9].log; do
  echo "$(basename $f .log) $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), round(d["value"]/1e6,2), round(d["scored_pairs_per_sec"]/1e6,1), round(d.get("configs1",{}).get("kernel_pairs_per_sec",0)/1e6,1))')"
done > $R/summary.txt
