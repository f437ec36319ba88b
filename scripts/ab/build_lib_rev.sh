#!/bin/bash
# build_lib_rev.sh NAME REV : libhdisort built from the sources of git revision REV
# -> mb/NAME/libhdisort.so (A/B runs via HD_LIB_PATH, e.g. scripts/ab/c4_ab.sh)
export HD_AB=1  # the A/B switches below are read only with this opt-in
set -e
NAME=$1; REV=$2
D=/root/repo/mb/$NAME
rm -rf $D; mkdir -p $D/src
git -C /root/repo archive "$REV" pyharp_amd/csrc include | tar -x -C $D/src
objs=""
for f in $D/src/pyharp_amd/csrc/*.hip $D/src/pyharp_amd/csrc/*.cpp; do
  s=$(basename $f)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -x hip -c $f -o $D/$s.o &
  objs="$objs $D/$s.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libhdisort.so $objs -lz
rm -rf $D/*.o $D/src
