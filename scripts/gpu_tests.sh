#!/bin/bash
# GPU parity suite only (one pytest process, per-test timeout).
#   gpurun --timeout 600 -- bash scripts/gpu_tests.sh TAG [pytest selectors...]
set -e -o pipefail
TAG=${1:-tests}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
SEL=${@:-tests}
echo "[tests] $(date +%T) pytest -m gpu $SEL"
timeout -k 10 540 python -u -m pytest $SEL -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
