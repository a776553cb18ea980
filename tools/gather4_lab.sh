#!/bin/bash
# Build gather4_lab variants (on this container) into tools/lab_bin/:
#   gather4_<SPW>_<WAVES>
set -e
cd "$(dirname "$0")"
mkdir -p lab_bin
for v in ${VARIANTS:-"8 8192" "4 8192" "8 4096" "4 16384"}; do
  set -- $v
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -Wno-unused-value -Wno-unused-result \
    -DGC_V4_SPW=$1 -DGC_V4_WAVES=$2 gather4_lab.hip -o lab_bin/gather4_$1_$2 &
done
wait
