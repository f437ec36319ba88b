#!/bin/bash
# build_lib_variant.sh NAME SED_EXPR FILE : libhdisort built from the in-tree sources with one
# sed edit applied to pyharp_amd/csrc/FILE -> mb/NAME/libhdisort.so (A/B runs via HD_LIB_PATH)
export HD_AB=1  # the A/B switches below are read only with this opt-in
set -e
NAME=$1; EXPR=$2; FILE=$3
D=/root/repo/mb/$NAME
rm -rf $D; mkdir -p $D/pyharp_amd/csrc $D/include/harp_amd
cp /root/repo/pyharp_amd/csrc/*.hip /root/repo/pyharp_amd/csrc/*.cpp /root/repo/pyharp_amd/csrc/*.hpp $D/pyharp_amd/csrc/
cp /root/repo/include/*.h $D/include/; cp /root/repo/include/harp_amd/*.hpp $D/include/harp_amd/
sed -i "$EXPR" $D/pyharp_amd/csrc/$FILE
grep -c "" $D/pyharp_amd/csrc/$FILE > /dev/null
objs=""
for s in hd_kernels.hip hd_team.hip hd_team_mfma.hip hd_rad.hip hd_rad_wide.hip hd_harp.hip hd_api.cpp hd_ncread.cpp; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -x hip -c $D/pyharp_amd/csrc/$s -o $D/$s.o &
  objs="$objs $D/$s.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libhdisort.so $objs -lz
rm -f $D/*.o
rm -rf $D/pyharp_amd $D/include
