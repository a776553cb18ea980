#!/bin/bash
# Build gemm_lab variants (on this container) into tools/lab_bin/:
#   VARIANTS="waves:rb:depth ..."  MODES="0 1 2 ..." (NT_LAB_MODE bits, see gemm_nt.hip)
set -e
cd "$(dirname "$0")"
mkdir -p lab_bin
for v in ${VARIANTS:-8:2:8}; do
  IFS=: read w r d <<< "$v"
  for m in ${MODES:-0}; do
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -Wno-unused-value -Wno-unused-result \
      -DNT_WAVES=$w -DNT_RB=$r -DNT_DEPTH=$d -DNT_LAB_MODE=$m $EXTRA gemm_lab.hip \
      -o lab_bin/gemm_lab_${w}_${r}_${d}_$m$SUFFIX &
  done
done
wait
