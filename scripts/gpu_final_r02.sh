#!/bin/bash
# Round-2 final tree: the whole GPU test suite, then the round-2 profile set.
#   gpurun --timeout 1200 -- bash scripts/gpu_final_r02.sh TAG
set -e -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
echo "[final] $(date +%T) pytest -m gpu"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
echo "[final] $(date +%T) smoke"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
cat "$OUT/smoke.log"
bash scripts/gpu_round2.sh "$TAG/r2"
echo "[final] $(date +%T) timeline c4"
timeout -k 10 180 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err"
cp "$(find "$OUT/trace" -name '*kernel_trace.csv' | head -1)" "$OUT/kernel_trace_c4.csv"
echo "[final] $(date +%T) done"
