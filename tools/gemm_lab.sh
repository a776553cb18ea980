#!/bin/bash
# Build gemm_lab for each NT_LAB_MODE (on this container) into tools/lab_bin/.
set -e
cd "$(dirname "$0")"
mkdir -p lab_bin
for m in ${MODES:-0 1 2 3 4 5}; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -Wno-unused-value -Wno-unused-result -DNT_LAB_MODE=$m gemm_lab.hip -o lab_bin/gemm_lab_$m &
done
wait
