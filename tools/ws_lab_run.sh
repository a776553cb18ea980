#!/bin/bash
# Run the gemm_ws lab binaries (tools/lab_bin/ws_lab_*) for every epilogue on
# the GPU box: bit-identity check against gemm_nt + timing at cfg3 shape.
set -o pipefail
mkdir -p gpurun_out
for b in ${BINS:-tools/lab_bin/ws_lab_*}; do
  for e in ${EPIS:-0 1 2 3 4 5}; do
    echo "== $b epi $e"
    timeout -k 5 60 $b 131072 512 512 $e 1 || exit 1
  done
done
