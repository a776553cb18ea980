#!/bin/bash
# Build tools/lab_bin/libdcnr_<name>.so with csrc/<file>.hip taken from a git
# revision (default HEAD) and every other object from the current build: an
# A/B partner for a change to one source file.
#   bash tools/lab_head.sh <name> <file.hip> [rev]
set -e
cd "$(dirname "$0")/.."
C=hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd/csrc
B=hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd/build
make -s -C $C
mkdir -p tools/lab_bin/src
name=$1; f=$2; rev=${3:-HEAD}
git show $rev:$C/$f > tools/lab_bin/src/${name}_$f
extra=""
[ "$f" = tower.hip ] && extra="-mllvm -amdgpu-mfma-vgpr-form"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $extra -I$C -c tools/lab_bin/src/${name}_$f -o tools/lab_bin/src/${name}.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/lab_bin/libdcnr_$name.so \
  $(ls $B/*.o | grep -v "/${f%.hip}.o\$") tools/lab_bin/src/${name}.o
echo built tools/lab_bin/libdcnr_$name.so
