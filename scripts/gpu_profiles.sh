#!/bin/bash
# Round profiles: bench lines for every config + rocprofv3 kernel stats (C4, C5) + PMC HBM bytes (C4).
set -e -o pipefail
TAG=${1:-prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
echo "[prof] $(date +%T) bench c4"
timeout -k 10 300 python bench.py > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err"
cat "$OUT/bench_c4.json"
echo "[prof] $(date +%T) bench c4 planck"
timeout -k 10 300 python bench.py --planck --no-cpu-baseline > "$OUT/bench_c4_planck.json" 2> "$OUT/bench_c4_planck.err"
for c in c5 c1 c3; do
  echo "[prof] $(date +%T) bench $c"
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err"
done
echo "[prof] $(date +%T) bench c1 graph"
timeout -k 10 300 python bench.py --config c1 --graph --steps 50 --warmup 5 > "$OUT/bench_c1_graph.json" 2> "$OUT/bench_c1_graph.err"
echo "[prof] $(date +%T) rocprof c4"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c4" -o kt --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > "$OUT/prof_c4.json" 2> "$OUT/prof_c4.err"
echo "[prof] $(date +%T) rocprof c5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c5" -o kt --output-format csv -- \
    python3 bench.py --config c5 --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/prof_c5.json" 2> "$OUT/prof_c5.err"
echo "[prof] $(date +%T) pmc"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o pmc --output-format csv -- \
    python3 scripts/pmc_run.py > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_write" -o pmc --output-format csv -- \
    python3 scripts/pmc_run.py > "$OUT/pmc_write.log" 2>&1
echo "[prof] $(date +%T) done"
