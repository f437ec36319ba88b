#!/bin/bash
# LDS-prefetch sweep: parity tests of the in-tree library, then A/B of C4 and the 8-GPU rank shape
# against the plain sweep (mb/nolds) and the early-S~- variant (mb/smearly).
#   gpurun --timeout 900 -- bash scripts/gpu_sweep_ab.sh TAG
set -e -o pipefail
TAG=${1:-sweep_ab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_band.py tests/test_gpu_concurrency.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for cfg in "c4:" "g8:--ngpoint 8" "g16:--ngpoint 16"; do
  name=${cfg%%:*}; args=${cfg#*:}
  for v in cur nolds smearly cur nolds; do
    if [ "$v" = cur ]; then unset HD_LIB_PATH; else export HD_LIB_PATH=$PWD/mb/$v/libhdisort.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 $args > "$OUT/${name}_$v.json" 2> "$OUT/${name}_$v.err"
    python -c "import json; d=json.load(open('$OUT/${name}_$v.json')); p=d['path_roofline']; print('$name $v', d['value'], d['ms_per_step'], 'layer', d['roofline']['avg_launch_ms'], 'sweep_ms/step', p.get('sweep_ms_per_step'))"
  done
done
echo done
