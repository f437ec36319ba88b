#!/bin/bash
# Small-shape A/B of library variants mb/<name> ("cur" = in-tree): C1, C3, the C5 and C4
# 8-GPU rank shapes, interleaved in the order given (bench.py --no-extra --no-cpu-baseline):
#   gpurun -- bash scripts/ab/shapes_ab.sh TAG v1 v2 v1 v2 ...
set -e -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
n=0
for v in "$@"; do
  n=$((n+1))
  if [ $v = cur ]; then unset HD_LIB_PATH; else export HD_LIB_PATH=$PWD/mb/$v/libhdisort.so; fi
  for shape in c1 c3 c5g8 c4g8; do
    case $shape in
      c1) a="--config c1 --steps 50 --warmup 5" ;;
      c3) a="--config c3 --steps 50 --warmup 5" ;;
      c5g8) a="--config c5 --ngpoint 8 --steps 10 --warmup 2" ;;
      c4g8) a="--config c4 --ngpoint 8 --steps 10 --warmup 2" ;;
    esac
    timeout -k 10 300 python bench.py $a --no-extra --no-cpu-baseline > $OUT/${shape}_${v}_$n.json 2> $OUT/${shape}_${v}_$n.err
    python -c "import json; d=json.load(open('$OUT/${shape}_${v}_$n.json')); print('$shape $v', d['value'], d['ms_per_step'])"
  done
done
