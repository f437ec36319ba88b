#!/bin/bash
# build_variant.sh NAME HD_DEVICE_HPP : libhdisort built with an alternative hd_device.hpp -> mb/NAME/libhdisort.so
set -e
NAME=$1; HDR=$2
D=/root/repo/mb/$NAME
rm -rf $D; mkdir -p $D/x/csrc $D/include
cp /root/repo/pyharp_amd/csrc/* $D/x/csrc/; cp /root/repo/include/*.h $D/include/
cp $HDR $D/x/csrc/hd_device.hpp
rm -f $D/x/csrc/*.o
objs=""
for s in hd_kernels.hip hd_team.hip hd_rad.hip hd_harp.hip hd_api.cpp; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -x hip -c $D/x/csrc/$s -o $D/$s.o &
  objs="$objs $D/$s.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libhdisort.so $objs
rm -f $D/*.o
