#!/bin/bash
# C5 (and its 8-GPU rank shape g8: --ngpoint 8) A/B of library variants mb/<name> ("cur" = in-tree),
# after the team-path parity tests on each variant:
#   gpurun -- bash scripts/ab/c5_ab.sh TAG v1 v2 v1 v2 ...
set -e -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in $(echo "$@" | tr ' ' '\n' | sort -u); do
  if [ $v = cur ]; then unset HD_LIB_PATH; else export HD_LIB_PATH=$PWD/mb/$v/libhdisort.so; fi
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_band.py tests/test_gpu_physics.py -m gpu -x -q --timeout 300 --timeout-method thread -k "18 or 20 or 22 or 24 or 26 or 28 or 30 or 32 or aerosol or c5" > $OUT/pytest_$v.log 2>&1 || { tail -30 $OUT/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $OUT/pytest_$v.log)"
done
n=0
for v in "$@"; do
  n=$((n+1))
  if [ $v = cur ]; then unset HD_LIB_PATH; else export HD_LIB_PATH=$PWD/mb/$v/libhdisort.so; fi
  for shape in c5 g8; do
    a=""; [ $shape = g8 ] && a="--ngpoint 8"
    timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 2 --no-extra --no-cpu-baseline $a > $OUT/${shape}_${v}_$n.json 2> $OUT/${shape}_${v}_$n.err
    python -c "import json; d=json.load(open('$OUT/${shape}_${v}_$n.json')); p=d['path_roofline']; print('$shape $v', d['value'], d['ms_per_step'], 'layer', p['layer_ms_per_step'], 'sweep', p['sweep_ms_per_step'], 'dev', d.get('max_rel_err_vs_cpu_restatement'))"
  done
done
