#!/bin/bash
# A/B: bench.py (C4, no CPU baseline) for each library variant given as mb/<name>/libhdisort.so ("cur" = in-tree)
export HD_AB=1  # the A/B switches below are read only with this opt-in
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
for v in "$@"; do
  if [ "$v" = cur ]; then unset HD_LIB_PATH; else export HD_LIB_PATH=$PWD/mb/$v/libhdisort.so; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 $AB_ARGS > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err
  python -c "import json,sys; d=json.load(open('gpurun_out/ab/$v.json')); r=d['roofline']; p=d['path_roofline']; print('$v', d['value'], 'layer_launch_ms', r['avg_launch_ms'], 'layer', p['layer_ms_per_step'], 'sweep', p['sweep_ms_per_step'])"
done
