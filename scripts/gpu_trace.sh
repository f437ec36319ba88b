#!/bin/bash
# Kernel timeline of a bench step (rocprofv3 kernel trace with timestamps):
#   gpurun -- bash scripts/gpu_trace.sh TAG [bench args...]
set -e -o pipefail
TAG=${1:-trace}; shift || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$TAG
timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/$TAG/raw -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 "$@" > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
f=$(find gpurun_out/$TAG/raw -name "*kernel_trace.csv" | head -1)
cp "$f" gpurun_out/$TAG/kernel_trace.csv
echo ok
