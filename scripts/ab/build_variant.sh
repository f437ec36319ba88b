#!/bin/bash
# Build libhdisort.so with the A/B-only kernel variants (HD_AB_VARIANTS=1: the
# column kernel, the LDS-state nstr-16 sweep, the one-wave team sweep, the VALU team
# kernels, the per-angle radiance kernel at nstr <= 16 -- DESIGN.md section 9) and
# extra compile flags into ab_libs/libhdisort_NAME.so (for A/B runs on one box:
# HD_LIB_PATH=ab_libs/libhdisort_NAME.so python ...; their tests: scripts/ab/tests):
#   bash scripts/ab/build_variant.sh NAME -DFLAG=VALUE ...
export HD_AB=1  # the A/B switches below are read only with this opt-in
set -e
NAME=$1; shift
OUT=ab_libs/obj_$NAME; mkdir -p $OUT
C=pyharp_amd/csrc
for src in hd_kernels.hip hd_team.hip hd_team_mfma.hip hd_rad.hip hd_harp.hip hd_api.cpp hd_ncread.cpp hd_rad_wide.hip; do
  extra=""; [ $src = hd_team_mfma.hip ] && extra="-mllvm -disable-machine-licm"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -x hip -DHD_AB_VARIANTS=1 "$@" $extra -c $C/$src -o $OUT/$src.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ab_libs/libhdisort_$NAME.so $OUT/*.o -lz
rm -rf $OUT
echo ab_libs/libhdisort_$NAME.so
