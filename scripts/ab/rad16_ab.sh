#!/bin/bash
# nstr-16 radiance: default library against ab_libs variants (HD_LIB_PATH), alternating
#   gpurun -- bash scripts/ab/rad16_ab.sh TAG VARIANT...
export HD_AB=1  # the A/B switches below are read only with this opt-in
set -e -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  timeout -k 10 300 python scripts/bench_rad.py --nstr 16 --steps 5 --warmup 2 > $OUT/base_$r.json
  python -c "import json; d=json.load(open('$OUT/base_$r.json')); print('base', round(d['value']), d['max_rel_err_subsample'])"
  for v in "$@"; do
    HD_LIB_PATH=ab_libs/libhdisort_$v.so timeout -k 10 300 python scripts/bench_rad.py --nstr 16 --steps 5 --warmup 2 > $OUT/${v}_$r.json
    python -c "import json; d=json.load(open('$OUT/${v}_$r.json')); print('$v', round(d['value']), d['max_rel_err_subsample'])"
  done
done
