#!/bin/bash
# C4 / 8-GPU-rank-shape A/B of library variants (mb/<name>/libhdisort.so; "cur" = in-tree),
# after the register-path parity tests on every variant:
#   gpurun -- bash scripts/ab/c4_ab.sh TAG cur v1 cur v1 ...
export HD_AB=1  # the A/B switches below are read only with this opt-in
set -e -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in $(echo "$@" | tr ' ' '\n' | sort -u); do
  if [ $v = cur ]; then unset HD_LIB_PATH; else export HD_LIB_PATH=$PWD/mb/$v/libhdisort.so; fi
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_band.py tests/test_gpu_physics.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_$v.log 2>&1 || { tail -30 $OUT/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $OUT/pytest_$v.log)"
done
n=0
for v in "$@"; do
  n=$((n+1))
  unset HD_LIB_PATH
  if [ $v != cur ]; then export HD_LIB_PATH=$PWD/mb/$v/libhdisort.so; fi
  for shape in c4 g8; do
    a=""; [ $shape = g8 ] && a="--ngpoint 8"
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra $a > $OUT/${shape}_${v}_$n.json 2> $OUT/${shape}_${v}_$n.err
    python -c "import json; d=json.load(open('$OUT/${shape}_${v}_$n.json')); p=d['path_roofline']; print('$shape $v', d['value'], d['ms_per_step'], 'layer', p['layer_ms_per_step'], 'sweep', p['sweep_ms_per_step'], 'dev', d.get('max_rel_err_vs_cpu_restatement'))"
  done
done
