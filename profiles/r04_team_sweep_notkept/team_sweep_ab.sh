#!/bin/bash
# nstr-16 sweep in 8-lane teams (HD_SWEEP_TEAM=1) against the one-lane sweep:
# register-path parity tests with the team sweep, then C4 and the 8-GPU rank
# shape alternating the two (same box):
#   gpurun -- bash scripts/ab/team_sweep_ab.sh TAG [ROUNDS]
set -e -o pipefail
TAG=$1; ROUNDS=${2:-2}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
HD_SWEEP_TEAM=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_band.py tests/test_gpu_physics.py tests/test_gpu_host_abi.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_team.log 2>&1 || { tail -30 $OUT/pytest_team.log; exit 1; }
tail -1 $OUT/pytest_team.log
for r in $(seq $ROUNDS); do
  for v in 0 1; do
    for shape in c4 g8; do
      a=""; [ $shape = g8 ] && a="--ngpoint 8"
      HD_SWEEP_TEAM=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra $a > $OUT/${shape}_t${v}_$r.json 2> $OUT/${shape}_t${v}_$r.err
      python -c "import json; d=json.load(open('$OUT/${shape}_t${v}_$r.json')); p=d['path_roofline']; print('$shape team=$v', d['value'], d['ms_per_step'], 'layer', p['layer_ms_per_step'], 'sweep', p['sweep_ms_per_step'], 'sum', d['band_flux_sum'])"
    done
  done
done
# kernel timeline of one C4 step with the team sweep
HD_SWEEP_TEAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_t1 -o kt --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra > $OUT/stats_t1.json 2> $OUT/stats_t1.err
python scripts/trace_timeline.py $(ls $OUT/stats_t1/*/kt_kernel_trace.csv | head -1) > $OUT/timeline_t1.txt
head -30 $OUT/timeline_t1.txt
