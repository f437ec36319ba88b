#!/bin/bash
# Round-2 closing run on the final tree (GPU tests, smoke, default bench line), then an
# A/B of the Jacobi residual check (mb/chk: HD_JACOBI_CHECK=1) -- its parity tests and
# bench lines at C4, the 8-GPU rank shape and one 60 000-solve chunk.
#   gpurun --timeout 900 -- bash scripts/gpu_final_chk.sh TAG
set -e -o pipefail
TAG=${1:-final3}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
echo "[fc] $(date +%T) pytest -m gpu"
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
cat "$OUT/smoke.log"
timeout -k 10 300 python bench.py > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err"
cat "$OUT/bench_c4.json"
echo "[fc] $(date +%T) chk parity"
HD_LIB_PATH=$GRAFT_REPO_ROOT/mb/chk/libhdisort.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_physics.py tests/test_gpu_radiance.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_chk.log" 2>&1 || { tail -30 "$OUT/pytest_chk.log"; exit 1; }
tail -1 "$OUT/pytest_chk.log"
for rep in 1 2; do
  for cfg in "c4:" "g8:--ngpoint 8" "g6:--ngpoint 6"; do
    name=${cfg%%:*}; args=${cfg#*:}
    for lib in tree chk; do
      if [ $lib = tree ]; then unset HD_LIB_PATH; else export HD_LIB_PATH=$GRAFT_REPO_ROOT/mb/$lib/libhdisort.so; fi
      timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 $args > "$OUT/${name}_${lib}_$rep.json" 2> "$OUT/${name}_${lib}_$rep.err"
      python -c "import json; d=json.load(open('$OUT/${name}_${lib}_$rep.json')); print('$name $lib $rep', d['value'], d['ms_per_step'], d['roofline'].get('avg_launch_ms'))"
    done
    unset HD_LIB_PATH
  done
done
echo "[fc] $(date +%T) done"
