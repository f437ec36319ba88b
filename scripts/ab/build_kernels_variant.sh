#!/bin/bash
# build_kernels_variant.sh NAME SED_EXPR : libhdisort with one sed edit applied to hd_kernels.hip only
# -> mb/NAME/libhdisort.so (the other translation units are compiled once into mb/_objs and reused).
# A/B runs load it via HD_LIB_PATH (scripts/ab/ab.sh).
export HD_AB=1  # the A/B switches below are read only with this opt-in
set -e
NAME=$1; EXPR=$2
R=/root/repo; C=$R/pyharp_amd/csrc; O=$R/mb/_objs
mkdir -p $O
for s in hd_team.hip hd_team_mfma.hip hd_rad.hip hd_rad_wide.hip hd_harp.hip hd_api.cpp hd_ncread.cpp; do
  if [ ! -f $O/$s.o ] || [ $C/$s -nt $O/$s.o ]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -x hip -c $C/$s -o $O/$s.o &
  fi
done
wait
D=$R/mb/$NAME; rm -rf $D; mkdir -p $D
sed "$EXPR" $C/hd_kernels.hip > $C/_variant_$NAME.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -x hip -c $C/_variant_$NAME.hip -o $D/k.o
rm -f $C/_variant_$NAME.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libhdisort.so $D/k.o $O/*.o -lz
rm -f $D/k.o
