#!/bin/bash
# layer-stream priority A/B (HD_LAY_PRIORITY) on C5 and C4: gpurun -- bash scripts/ab/prio_ab.sh TAG
set -e -o pipefail
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for v in none high low; do
    for cfg in c5 c4; do
      HD_LAY_PRIORITY=$v timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-extra > $OUT/${cfg}_${v}_$r.json 2> $OUT/${cfg}_${v}_$r.err
      python -c "import json; d=json.load(open('$OUT/${cfg}_${v}_$r.json')); print('$cfg $v', d['value'], d['ms_per_step'])"
    done
  done
done
