#!/bin/bash
# Build mb/NAME/libhdisort.so from a variant of hd_kernels.hip (FILE), linking the
# other translation units from an object cache (OBJCACHE, default /tmp/objcache,
# filled by: bash scripts/ab/kvariant.sh --cache):
#   bash scripts/ab/kvariant.sh NAME FILE [extra hipcc flags]
set -e
C=pyharp_amd/csrc
CACHE=${OBJCACHE:-/tmp/objcache}
if [ "$1" = --cache ]; then
  mkdir -p $CACHE
  for src in hd_team.hip hd_team_mfma.hip hd_rad.hip hd_harp.hip hd_api.cpp hd_ncread.cpp hd_rad_wide.hip; do
    extra=""; [ $src = hd_team_mfma.hip ] && extra="-mllvm -disable-machine-licm"
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -x hip $extra -c $C/$src -o $CACHE/$src.o &
  done
  wait; exit 0
fi
NAME=$1; FILE=$2; shift 2
mkdir -p mb/$NAME
cp "$FILE" $C/hd_kernels_variant_tmp.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -x hip "$@" -c $C/hd_kernels_variant_tmp.hip -o mb/$NAME/k.o
rm -f $C/hd_kernels_variant_tmp.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o mb/$NAME/libhdisort.so mb/$NAME/k.o $CACHE/*.o -lz
rm mb/$NAME/k.o
echo mb/$NAME/libhdisort.so
