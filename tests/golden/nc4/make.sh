#!/bin/bash
# Regenerate the netCDF-4 fixtures with the image's HDF5 library (see make_nc4.c).
set -euo pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
gcc "$HERE/make_nc4.c" -I/opt/conda/include -L/opt/conda/lib -lhdf5_hl -lhdf5 \
    -Wl,-rpath,/opt/conda/lib -lm -o /tmp/make_nc4
/tmp/make_nc4 "$HERE"
ls -l "$HERE"/*.nc
