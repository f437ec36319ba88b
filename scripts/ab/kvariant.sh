#!/bin/bash
# Build mb/NAME/libhdisort.so with one translation unit replaced by a variant FILE
# (default TU hd_kernels.hip), linking the others from an object cache (OBJCACHE,
# default /tmp/objcache, filled from the tree by: bash scripts/ab/kvariant.sh --cache):
#   bash scripts/ab/kvariant.sh NAME FILE [TU] [extra hipcc flags]
set -e
C=pyharp_amd/csrc
CACHE=${OBJCACHE:-/tmp/objcache}
ALL="hd_kernels.hip hd_team.hip hd_team_mfma.hip hd_rad.hip hd_harp.hip hd_api.cpp hd_ncread.cpp hd_rad_wide.hip"
flags_of() { [ $1 = hd_team_mfma.hip ] && echo "-mllvm -disable-machine-licm"; }
if [ "$1" = --cache ]; then
  mkdir -p $CACHE
  for src in $ALL; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -x hip $(flags_of $src) -c $C/$src -o $CACHE/$src.o &
  done
  wait; exit 0
fi
NAME=$1; FILE=$2; TU=${3:-hd_kernels.hip}; shift 2; [ $# -gt 0 ] && shift
mkdir -p mb/$NAME
ext=${TU##*.}
cp "$FILE" $C/variant_tmp_$NAME.$ext
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -x hip $(flags_of $TU) "$@" -c $C/variant_tmp_$NAME.$ext -o mb/$NAME/v.o
rm -f $C/variant_tmp_$NAME.$ext
objs=""
for src in $ALL; do [ $src != $TU ] && objs="$objs $CACHE/$src.o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o mb/$NAME/libhdisort.so mb/$NAME/v.o $objs -lz
rm mb/$NAME/v.o
echo mb/$NAME/libhdisort.so
