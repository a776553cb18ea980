#!/bin/bash
# Build tools/lab_bin/libdcnr_<name>.so with a sed-edited copy of the current
# csrc/<file>.hip and every other object from the current build.
#   bash tools/lab_sed.sh <name> <file.hip> 'sed expr' ['sed expr' ...]
set -e
cd "$(dirname "$0")/.."
C=hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd/csrc
B=hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd/build
make -s -C $C
mkdir -p tools/lab_bin/src
name=$1; f=$2; shift 2
src=tools/lab_bin/src/${name}_$f
cp $C/$f $src
for e in "$@"; do sed -i "$e" $src; done
if cmp -s $C/$f $src; then echo "lab_sed: no edit applied" >&2; exit 1; fi
extra=""
[ "$f" = tower.hip ] && extra="-mllvm -amdgpu-mfma-vgpr-form"
[ "$f" = gemm_wsp.hip ] && extra="-mllvm -amdgpu-mfma-vgpr-form -fno-slp-vectorize"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $extra -I$C -c $src -o tools/lab_bin/src/${name}.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/lab_bin/libdcnr_$name.so \
  $(ls $B/*.o | grep -v "/${f%.hip}.o\$") tools/lab_bin/src/${name}.o
echo built tools/lab_bin/libdcnr_$name.so
