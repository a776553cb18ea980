#!/bin/bash
# lab: BIAS_STATS / BIAS tile rows, RESID_BN tile rows (1-bit masks)
mkdir -p gpurun_out
for b in tools/lab_bin/ws_lab_*; do
  for e in 0 3; do echo "== $b epi $e"; timeout -k 5 60 $b 131072 512 512 $e 1 || exit 1; done
  echo "== $b epi 4 hb1"; timeout -k 5 60 $b 131072 512 512 4 0 1 || exit 1
done
