#!/bin/bash
# C5 A/B of library variants (mb/<name>/libhdisort.so; "cur" = in-tree): team parity
# tests on each, then the C5 bench with the CPU-restatement comparison (max_rel_err).
#   gpurun -- bash scripts/ab/c5_ab.sh TAG cur v1 v2 ...
export HD_AB=1  # the A/B switches below are read only with this opt-in
set -e -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  unset HD_LIB_PATH
  if [ $v != cur ]; then export HD_LIB_PATH=$PWD/mb/$v/libhdisort.so; fi
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "18 or 20 or 22 or 24 or 26 or 28 or 30 or 32 or team or aerosol" > $OUT/pytest_$v.log 2>&1 || { tail -30 $OUT/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $OUT/pytest_$v.log)"
  OMP_NUM_THREADS=16 timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 > $OUT/c5_$v.json 2> $OUT/c5_$v.err
  python -c "import json; d=json.load(open('$OUT/c5_$v.json')); p=d['path_roofline']; print('$v', d['value'], d['ms_per_step'], 'layer', p['layer_ms_per_step'], 'sweep', p['sweep_ms_per_step'], 'err', d['max_rel_err_vs_cpu_restatement'])"
done
