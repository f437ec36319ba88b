#!/bin/bash
# A/B: how many of the last chunks' back-substitutions take the uncapped tail kernel
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tail2
for v in 1 2 3 1 2 3; do
  for cfg in "c4:" "g8:--ngpoint 8" "g16:--ngpoint 16" "g32:--ngpoint 32"; do
    name=${cfg%%:*}; args=${cfg#*:}
    HD_TAIL_LAST=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 $args > gpurun_out/tail2/${name}_$v.json 2> gpurun_out/tail2/${name}_$v.err
    python -c "import json; d=json.load(open('gpurun_out/tail2/${name}_$v.json')); print('$name tail_last=$v', d['value'], d['ms_per_step'])"
  done
done
