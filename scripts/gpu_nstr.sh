#!/bin/bash
# C5-shaped bench at every team-path nstr (spill check)
set -e -o pipefail
OUT=gpurun_out/${1:-nstr}
mkdir -p "$OUT"
for n in 18 20 24 28 30 32; do
  timeout -k 10 200 python bench.py --config c5 --nstr $n --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/c5_n$n.json" 2> "$OUT/c5_n$n.err"
  python -c "import json; d=json.load(open('$OUT/c5_n$n.json')); print($n, d['value'], d['path_roofline'])"
done
