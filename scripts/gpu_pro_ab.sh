#!/bin/bash
# Register-path prologue on its own stream: GPU tests on the in-tree library, then
# C4 / 8-GPU-rank-shape bench lines of tree, mb/old (prologue on the side stream) and
# the 1-Jacobi-sweep timing variants of both (mb/old_ms1, mb/new_ms1; wrong fluxes,
# timing only: what a cheaper layer kernel would buy under each schedule).
#   gpurun --timeout 900 -- bash scripts/gpu_pro_ab.sh TAG
set -e -o pipefail
TAG=${1:-pro}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
echo "[pro] $(date +%T) pytest -m gpu"
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for rep in 1 2; do
  for cfg in "c4:" "g8:--ngpoint 8" "g16:--ngpoint 16"; do
    name=${cfg%%:*}; args=${cfg#*:}
    for lib in tree old old_ms1 new_ms1; do
      if [ $lib = tree ]; then unset HD_LIB_PATH; else export HD_LIB_PATH=$GRAFT_REPO_ROOT/mb/$lib/libhdisort.so; fi
      timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 $args > "$OUT/${name}_${lib}_$rep.json" 2> "$OUT/${name}_${lib}_$rep.err"
      python -c "import json; d=json.load(open('$OUT/${name}_${lib}_$rep.json')); print('$name $lib $rep', d['value'], d['ms_per_step'], d['roofline'].get('avg_launch_ms'))"
    done
    unset HD_LIB_PATH
  done
done
echo "[pro] $(date +%T) done"
