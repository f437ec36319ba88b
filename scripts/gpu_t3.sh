#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/${1:-t3}
mkdir -p "$OUT"
timeout -k 10 600 python -m pytest tests -m gpu -x -q > "$OUT/pytest.log" 2>&1 || { tail -60 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 120 python examples/amars_sw.py > "$OUT/amars_sw.txt" 2>&1
head -4 "$OUT/amars_sw.txt"
