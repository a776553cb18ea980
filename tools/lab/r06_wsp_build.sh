#!/bin/bash
# Build tools/lab_bin/libdcnr_wsp<V>.so: the current library with the train
# forward's BIAS / BIAS_STATS GEMMs (256 < K <= 512) dispatched to
# tools/lab/gemm_wsp_lab.hip built with -DWSP_VAR=<V>.
#   bash tools/lab/r06_wsp_build.sh "0 1 2 3"
set -e
cd "$(dirname "$0")/../.."
C=hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd/csrc
B=hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd/build
make -s -C $C
S=tools/lab_bin/src; mkdir -p $S
cp $C/gemm_ws.hip $S/gemm_ws_wspdispatch.hip
sed -i 's|#include "dcnr_internal.h"|#include "dcnr_internal.h"\nnamespace dcnr { bool gemm_wsp_supported(int, int64_t, int64_t); dcnr_status gemm_wsp(int, const NtArgs\&, hipStream_t, int*); }|' $S/gemm_ws_wspdispatch.hip
sed -i 's|^  switch (epi) {|  if (gemm_wsp_supported(epi, a.K, a.N)) return gemm_wsp(epi, a, s, nparts);\n  switch (epi) {|' $S/gemm_ws_wspdispatch.hip
grep -q "return gemm_wsp(epi" $S/gemm_ws_wspdispatch.hip
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$C"
$H -c $S/gemm_ws_wspdispatch.hip -o $S/gemm_ws_wspdispatch.o
for v in $1; do
  $H -mllvm -amdgpu-mfma-vgpr-form -fno-slp-vectorize -DWSP_VAR=$v -c tools/lab/gemm_wsp_lab.hip -o $S/gemm_wsp_$v.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/lab_bin/libdcnr_wsp$v.so \
    $(ls $B/*.o | grep -v "/gemm_ws.o\$") $S/gemm_ws_wspdispatch.o $S/gemm_wsp_$v.o
  echo built tools/lab_bin/libdcnr_wsp$v.so
done
