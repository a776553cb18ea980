#!/bin/bash
# A/B of library builds on the train step (on the GPU box, repo root):
#   bash tools/ab_bench.sh <outdir> <rounds> v1 v2 ...   (tools/lab_bin/libdcnr_<v>.so)
# each round runs every variant once, alternating, so box drift hits all alike
set -o pipefail
OUT=$1; ROUNDS=$2; shift 2
mkdir -p $OUT
ROOT=$(pwd)
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    DCNR_LIB=$ROOT/tools/lab_bin/libdcnr_$v.so timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 \
        --no-cpu-baseline --no-serving --no-fp32 --no-zipf > $OUT/${v}_$r.log 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads(open('$OUT/${v}_$r.log').read().strip().split('\n')[-1]); print('$v', $r, round(d['ms_per_step'],4))" | tee -a $OUT/summary.txt
  done
done
