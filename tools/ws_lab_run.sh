#!/bin/bash
# Time the gemm_ws lab binaries (tools/lab_bin/ws_lab_*) on the GPU box for the
# epilogues in EPIS at the cfg3 shape.
set -o pipefail
for b in ${BINS:-tools/lab_bin/ws_lab_*}; do
  for e in ${EPIS:-0 1 2 3 4 5 6 7}; do
    timeout -k 5 60 $b 131072 512 512 $e || exit 1
  done
done
