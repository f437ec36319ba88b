#!/bin/bash
# A/B of an environment switch on the in-tree library: register-path parity tests
# with the switch at its first value, then C4 and the 8-GPU rank shape for each value.
#   gpurun -- bash scripts/ab/env_ab.sh TAG VAR v1 v2 [v1 v2 ...]
export HD_AB=1  # the A/B switches below are read only with this opt-in
set -e -o pipefail
TAG=$1; VAR=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
env $VAR=$1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_band.py tests/test_gpu_physics.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
n=0
for v in "$@"; do
  n=$((n+1))
  for shape in c4 g8; do
    a=""; [ $shape = g8 ] && a="--ngpoint 8"
    env $VAR=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline $a > $OUT/${shape}_${v}_$n.json 2> $OUT/${shape}_${v}_$n.err
    python -c "import json; d=json.load(open('$OUT/${shape}_${v}_$n.json')); p=d['path_roofline']; print('$shape $VAR=$v', d['value'], d['ms_per_step'], 'layer', p['layer_ms_per_step'], 'sweep', p['sweep_ms_per_step'])"
  done
done
