#!/bin/bash
# Jacobi warm-start A/B (round 3): the in-tree library (warm start on) against a
# baseline variant: register + team parity tests on the in-tree library, then C4,
# the 8-GPU rank shape and C5, alternating.
#   gpurun -- bash scripts/ab/warm_ab.sh TAG BASE
export HD_AB=1  # the A/B switches below are read only with this opt-in
set -e -o pipefail
TAG=$1; BASE=$2
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_band.py tests/test_gpu_physics.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in cur $BASE cur $BASE; do
  unset HD_LIB_PATH
  if [ $v != cur ]; then export HD_LIB_PATH=$PWD/mb/$v/libhdisort.so; fi
  for shape in c4 g8 c5; do
    a="--steps 10 --warmup 3"; [ $shape = g8 ] && a="$a --ngpoint 8"; [ $shape = c5 ] && a="--config c5 --steps 4 --warmup 1"
    timeout -k 10 300 python bench.py $a --no-cpu-baseline > $OUT/${shape}_$v.json 2> $OUT/${shape}_$v.err
    python -c "import json; d=json.load(open('$OUT/${shape}_$v.json')); p=d['path_roofline']; print('$shape $v', d['value'], d['ms_per_step'], 'layer', p['layer_ms_per_step'], 'sweep', p['sweep_ms_per_step'], 'err', d.get('max_rel_err_vs_cpu_restatement'))"
  done
done
