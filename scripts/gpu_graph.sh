#!/bin/bash
set -e -o pipefail
OUT=gpurun_out/${1:-graph}
mkdir -p "$OUT"
for c in c1 c3 c4; do
  for g in "" "--graph"; do
    timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline $g > "$OUT/$c$g.json" 2> "$OUT/$c$g.err" || { tail -20 "$OUT/$c$g.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/$c$g.json')); print('$c', '$g', d['value'], d['ms_per_step'], d['path_roofline'])"
  done
done
