#!/bin/bash
# repeat the two bit-identity tests of the embedding backward per library
set -o pipefail
R=gpurun_out/$1; mkdir -p $R
for v in $2; do
  for i in 1 2 3; do
    if [ $v = base ]; then unset DCNR_LIB; else export DCNR_LIB=$PWD/tools/lab_bin/libdcnr_$v.so; fi
    timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread \
      tests/test_embed_bwd_gpu.py -k "accumulate or side_stream or deterministic" > $R/${v}_$i.log 2>&1
    echo "$v $i: $(tail -n 1 $R/${v}_$i.log)" >> $R/summary.txt
  done
done
