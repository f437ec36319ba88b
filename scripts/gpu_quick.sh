#!/bin/bash
# Quick GPU iteration: parity tests, then the C4 bench line (no CPU baseline).
#   gpurun --timeout 600 -- bash scripts/gpu_quick.sh TAG [bench args...]
set -e -o pipefail
TAG=${1:-quick}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
echo "[quick] $(date +%T) pytest -m gpu"
timeout -k 10 420 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
echo "[quick] $(date +%T) bench"
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
