#!/bin/bash
# Round-2 profile set: C4 bench (CPU baseline), kernel trace + stats (C4, C5),
# PMC HBM bytes of one C4 chunk on the fused path, and the other bench shapes.
#   gpurun --timeout 1200 -- bash scripts/gpu_round2.sh TAG
set -e -o pipefail
TAG=${1:-r2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
echo "[r2] $(date +%T) bench c4"
timeout -k 10 300 python bench.py > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err"
cat "$OUT/bench_c4.json"
echo "[r2] $(date +%T) rocprof c4"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c4" -o kt --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > "$OUT/prof_c4.json" 2> "$OUT/prof_c4.err"
echo "[r2] $(date +%T) rocprof c5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c5" -o kt --output-format csv -- \
    python3 bench.py --config c5 --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/prof_c5.json" 2> "$OUT/prof_c5.err"
echo "[r2] $(date +%T) pmc"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o pmc --output-format csv -- \
    python3 scripts/pmc_run.py > "$OUT/pmc_fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_write" -o pmc --output-format csv -- \
    python3 scripts/pmc_run.py > "$OUT/pmc_write.log" 2>&1
for c in c5 c3l c1; do
  echo "[r2] $(date +%T) bench $c"
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err"
done
echo "[r2] $(date +%T) bench g8/g16/g32 (per-rank shard shapes)"
for g in 8 16 32; do
  timeout -k 10 300 python bench.py --ngpoint $g --no-cpu-baseline > "$OUT/bench_g$g.json" 2> "$OUT/bench_g$g.err"
done
echo "[r2] $(date +%T) done"
