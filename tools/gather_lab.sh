#!/bin/bash
# Build gather_lab for each GC_LAB_MODE (on this container) into tools/lab_bin/.
set -e
cd "$(dirname "$0")"
mkdir -p lab_bin
for m in ${MODES:-0 1 2 3 4 7}; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -Wno-unused-value -Wno-unused-result -DGC_LAB_MODE=$m gather_lab.hip -o lab_bin/gather_lab_$m &
done
wait
