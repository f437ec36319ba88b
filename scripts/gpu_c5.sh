#!/bin/bash
# C5 (nstr=32) bench + kernel stats on the GPU box.
set -e -o pipefail
OUT=gpurun_out/${1:-c5}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[c5] $(date +%T) bench c5"
timeout -k 10 400 python bench.py --config c5 --steps 3 --warmup 1 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" || { tail -20 "$OUT/bench_c5.err"; exit 1; }
cat "$OUT/bench_c5.json"
echo "[c5] $(date +%T) rocprof c5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o kt --output-format csv -- \
    python3 bench.py --config c5 --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/prof_c5.json" 2> "$OUT/prof.err"
cat "$OUT/prof_c5.json"
head -4 "$OUT/prof/kt_kernel_stats.csv" | cut -c1-160
