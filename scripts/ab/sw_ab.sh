export HD_AB=1  # the A/B switches below are read only with this opt-in
set -e -o pipefail
OUT=gpurun_out/r2s3_swab; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_band.py -m gpu -x -q --timeout 120 --timeout-method thread -k "18 or 20 or 22 or 24 or 26 or 28 or 30 or 32 or team or aerosol or band" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in cur sw1 valu; do
  unset HD_LIB_PATH HD_TEAM_SWEEP
  if [ $v = sw1 ]; then export HD_LIB_PATH=$PWD/mb/sw1/libhdisort.so; fi
  if [ $v = valu ]; then export HD_TEAM_SWEEP=valu; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --config c5 --steps 3 --warmup 1 > $OUT/c5_$v.json 2> $OUT/c5_$v.err
  python -c "import json; d=json.load(open('$OUT/c5_$v.json')); p=d['path_roofline']; print('$v', d['value'], d['ms_per_step'], 'layer', p['layer_ms_per_step'], 'sweep', p['sweep_ms_per_step'])"
done
