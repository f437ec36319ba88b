#!/bin/bash
# chunk-size sweep after the tail-kernel rule (<= 3 chunks: every back-substitution uncapped)
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/chunk2
for cfg in "g8_auto:--ngpoint 8" "g8_26667:--ngpoint 8 --chunk 26667" "g8_20000:--ngpoint 8 --chunk 20000" "g16_auto:--ngpoint 16" "g16_40000:--ngpoint 16 --chunk 40000" "c4_auto:" "c4_80000:--chunk 80000" "c4_128000:--chunk 128000" "c4_213334:--chunk 213334"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 8 --warmup 2 $args > gpurun_out/chunk2/$name.json 2> gpurun_out/chunk2/$name.err
  python -c "import json; d=json.load(open('gpurun_out/chunk2/$name.json')); print('$name', d['value'], d['ms_per_step'])"
done
