#!/bin/bash
# Compile the C++ drop-in checks against the container's libtorch (ROCm build)
# and the in-tree libhdisort.so.  Outputs: tests/cpp/disort_dropin, tests/cpp/amars_sw_dropin,
# tests/cpp/disort_rad_dropin, tests/cpp/amars_lw_dropin, tests/cpp/radiation_band_swap,
# tests/cpp/flags_check,
# and the plain-C host-array caller tests/cpp/host_abi (gcc, no torch)
set -euo pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/../.." && pwd)
TORCH=$(python -c "import torch, os; print(os.path.dirname(torch.__file__))")
ABI=$(python -c "import torch; print(int(torch._C._GLIBCXX_USE_CXX11_ABI))")
build() {
  /opt/rocm/bin/hipcc -O2 -std=c++17 -D_GLIBCXX_USE_CXX11_ABI=$ABI -D__HIP_PLATFORM_AMD__ -DUSE_ROCM \
    -I"$ROOT/include" -I"$TORCH/include" -I"$TORCH/include/torch/csrc/api/include" \
    "$HERE/$1.cpp" -o "$HERE/$1" \
    -L"$TORCH/lib" -Wl,-rpath,"$TORCH/lib" -ltorch -ltorch_cpu -lc10 -ltorch_hip -lc10_hip \
    -L"$ROOT/pyharp_amd" -Wl,-rpath,'$ORIGIN/../../pyharp_amd' -lhdisort -lz
}
build disort_dropin &
build amars_sw_dropin &
build disort_rad_dropin &
build amars_lw_dropin &
build radiation_band_swap &
build flags_check &
gcc -O2 -std=c99 -I"$ROOT/include" "$HERE/host_abi.c" -o "$HERE/host_abi" -lm \
  -L"$ROOT/pyharp_amd" -Wl,-rpath,'$ORIGIN/../../pyharp_amd' -lhdisort &
wait %1 && wait %2 && wait %3 && wait %4 && wait %5 && wait %6 && wait %7
