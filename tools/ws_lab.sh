#!/bin/bash
# Build ws_lab for each WS_LAB_MODE (on this container) into tools/lab_bin/.
set -e
cd "$(dirname "$0")"
D=${OUTDIR:-lab_bin}
mkdir -p $D
C=../hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd/csrc
for m in ${MODES:-0}; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -Wno-unused-result -Wno-unused-value -DWS_LAB_MODE=$m \
    $EXTRA ws_lab.hip $C/gemm_ws.hip -o $D/ws_lab_$m$SUFFIX &
done
wait
