#!/bin/bash
# Last-chunk layer segments (HD_LAST_SEGMENTS): register-path parity tests with 4
# segments, then C4 and the 8-GPU rank shape at 1 / 2 / 4 / 8 segments, twice.
set -e -o pipefail
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
HD_LAST_SEGMENTS=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_band.py tests/test_gpu_physics.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
  for n in 1 2 4 8; do
    for shape in c4 g8; do
      a=""; [ $shape = g8 ] && a="--ngpoint 8"
      HD_LAST_SEGMENTS=$n timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline $a > $OUT/${shape}_s${n}_$rep.json 2> $OUT/${shape}_s${n}_$rep.err
      python -c "import json; d=json.load(open('$OUT/${shape}_s${n}_$rep.json')); print('$shape seg $n', d['value'], d['ms_per_step'])"
    done
  done
done
