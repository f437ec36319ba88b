#!/bin/bash
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c5chunk
for ch in 0 8000 10667 12800 0 8000 6400; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --config c5 --steps 4 --warmup 1 --chunk $ch > gpurun_out/c5chunk/c$ch.json 2> gpurun_out/c5chunk/c$ch.err
  python -c "import json; d=json.load(open('gpurun_out/c5chunk/c$ch.json')); print('chunk $ch', d['value'], d['ms_per_step'], 'layer', d['roofline']['avg_launch_ms'])"
done
