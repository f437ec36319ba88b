#!/bin/bash
# radiance throughput against the chunk size (solves per chunk): scripts/bench_rad.py
#   gpurun -- bash scripts/ab/rad_chunk_ab.sh TAG
export HD_AB=1  # the A/B switches below are read only with this opt-in
set -e -o pipefail
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for n in 16 32; do
  for ch in 0 2000 1000 500 250; do
    timeout -k 10 300 python scripts/bench_rad.py --nstr $n --steps 3 --warmup 1 --chunk $ch > $OUT/rad_n${n}_c${ch}.json
    python -c "import json; d=json.load(open('$OUT/rad_n${n}_c${ch}.json')); print('nstr $n chunk $ch', round(d['value']), round(d['ms_per_step'],1), d['max_rel_err_subsample'])"
  done
done
