#!/bin/bash
# Build libdcnr variants with sed-edited copies of csrc/tower.hip into
# tools/lab_bin/libdcnr_tw_<name>.so (here, on the CPU container), e.g.
#   bash tools/tower_lab.sh s4 's/TW_NSLOT = 3;/TW_NSLOT = 4;/'
# then on the box: DCNR_LIB=$PWD/tools/lab_bin/libdcnr_tw_s4.so python tools/tower_probe.py
set -e
cd "$(dirname "$0")/.."
C=hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd/csrc
B=hybrid-hotel-recommendation-system-based-on-friends-recommendations_amd/build
make -s -C $C
mkdir -p tools/lab_bin/twsrc
name=$1; shift
src=tools/lab_bin/twsrc/tower_$name.hip
cp $C/tower.hip $src
for e in "$@"; do sed -i "$e" $src; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC ${TWFLAGS:-} -I$C -c $src -o tools/lab_bin/twsrc/tower_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/lab_bin/libdcnr_tw_$name.so \
  $(ls $B/*.o | grep -v '/tower.o$') tools/lab_bin/twsrc/tower_$name.o
echo built tools/lab_bin/libdcnr_tw_$name.so
