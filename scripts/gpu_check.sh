#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats, PMC passes.
#   gpurun --timeout 1100 -- bash scripts/gpu_check.sh TAG [bench args...]
# Every GPU step has its own time limit; steps are chained so the first failure ends the run.
set -e -o pipefail
TAG=${1:-run}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
echo "[gpu_check] $(date +%T) pytest -m gpu"
timeout -k 10 420 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
echo "[gpu_check] $(date +%T) smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
cat "$OUT/smoke.log"
echo "[gpu_check] $(date +%T) bench"
timeout -k 10 300 python bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
echo "[gpu_check] $(date +%T) bench planck"
timeout -k 10 300 python bench.py --planck --no-cpu-baseline "$@" > "$OUT/bench_planck.json" 2> "$OUT/bench_planck.err"
cat "$OUT/bench_planck.json"
echo "[gpu_check] $(date +%T) rocprofv3 kernel stats"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o kt --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 "$@" > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
cat "$OUT/prof_bench.json"
echo "[gpu_check] $(date +%T) pmc FETCH_SIZE"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o pmc --output-format csv -- \
    python3 scripts/pmc_run.py > "$OUT/pmc_fetch.log" 2>&1
echo "[gpu_check] $(date +%T) pmc WRITE_SIZE"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_write" -o pmc --output-format csv -- \
    python3 scripts/pmc_run.py > "$OUT/pmc_write.log" 2>&1
echo "[gpu_check] $(date +%T) done"
find "$OUT" -name "*.csv" | head -20
