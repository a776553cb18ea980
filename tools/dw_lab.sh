#!/bin/bash
# Build dw_lab for each DW_LAB_MODE (on this container) into tools/lab_bin/; run on the box:
#   for b in tools/lab_bin/dw_lab_*; do $b; done
set -e
cd "$(dirname "$0")"
mkdir -p lab_bin
for m in ${MODES:-0 1 2 4}; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -Wno-unused-result -Wno-unused-value -DDW_LAB_MODE=$m \
    $EXTRA dw_lab.hip -o lab_bin/dw_lab_$m$SUFFIX &
done
wait
