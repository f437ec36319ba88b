#!/bin/bash
# build_lib_ref.sh NAME GITREF : libhdisort from the sources of commit GITREF -> mb/NAME/libhdisort.so
# (A/B of the working tree against a commit, loaded via HD_LIB_PATH)
export HD_AB=1  # the A/B switches below are read only with this opt-in
set -e
NAME=$1; REF=$2
D=/root/repo/mb/$NAME
rm -rf $D; mkdir -p $D/src
git -C /root/repo archive "$REF" pyharp_amd/csrc include | tar -x -C $D/src
objs=""
for s in hd_kernels.hip hd_team.hip hd_team_mfma.hip hd_rad.hip hd_rad_wide.hip hd_harp.hip hd_api.cpp hd_ncread.cpp; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -x hip -c $D/src/pyharp_amd/csrc/$s -o $D/$s.o &
  objs="$objs $D/$s.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libhdisort.so $objs -lz
rm -rf $D/*.o $D/src
