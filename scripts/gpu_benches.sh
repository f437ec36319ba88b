#!/bin/bash
# Bench lines for several configs on one box, one timed step each (chained with &&).
#   gpurun --timeout 900 -- bash scripts/gpu_benches.sh TAG "c4" "c1" "c3 --no-cpu-baseline" ...
# Each quoted argument is a bench.py argument list after --config; output
# gpurun_out/TAG/bench_<n>.json (+ .err).
set -e -o pipefail
TAG=${1:-benches}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
i=0
for a in "$@"; do
  i=$((i+1))
  echo "[benches] $(date +%T) bench --config $a"
  timeout -k 10 300 python bench.py --config $a > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err" || { tail -20 "$OUT/bench_$i.err"; exit 1; }
  cat "$OUT/bench_$i.json"
done
