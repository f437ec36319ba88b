#!/bin/bash
# Team-path A/B (nstr 18..32): team parity tests on the in-tree library, the GPU
# Jacobi sweep counts at nstr 32, then C5 (with the CPU-restatement deviation on the
# bench sample) for the in-tree library and a baseline variant, alternating.
#   gpurun -- bash scripts/ab/team_ab.sh TAG BASE
export HD_AB=1  # the A/B switches below are read only with this opt-in
set -e -o pipefail
TAG=$1; BASE=$2
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_physics.py tests/test_gpu_radiance.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python scripts/micro/sweep_count.py 32 | tee $OUT/sweeps.txt
for v in cur $BASE cur $BASE; do
  unset HD_LIB_PATH
  if [ $v != cur ]; then export HD_LIB_PATH=$PWD/mb/$v/libhdisort.so; fi
  OMP_NUM_THREADS=16 timeout -k 10 300 python bench.py --config c5 --steps 4 --warmup 1 > $OUT/c5_$v.json 2> $OUT/c5_$v.err
  python -c "import json; d=json.load(open('$OUT/c5_$v.json')); p=d['path_roofline']; print('c5 $v', d['value'], d['ms_per_step'], 'layer', p['layer_ms_per_step'], 'sweep', p['sweep_ms_per_step'], 'err', d.get('max_rel_err_vs_cpu_restatement'))"
done
