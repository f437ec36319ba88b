#!/bin/bash
# C5 team sweep: lean (two waves per SIMD, HD_TEAM_SWEEP_LEAN=1) against the
# one-wave sweep.  Team-path parity tests with the lean sweep, the bitwise test,
# then C5 / C5s alternating the two (same box), and a C5 timeline with the lean sweep:
#   gpurun -- bash scripts/ab/lean_ab.sh TAG [ROUNDS]
export HD_AB=1  # the A/B switches below are read only with this opt-in
set -e -o pipefail
TAG=$1; ROUNDS=${2:-2}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
HD_TEAM_SWEEP_LEAN=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_lean_sweep.py tests/test_gpu_parity.py tests/test_gpu_warm.py tests/test_gpu_physics.py -m gpu -x -q --timeout 300 --timeout-method thread -k "lean or 18 or 20 or 22 or 24 or 26 or 28 or 30 or 32 or aerosol or c5 or warm" > $OUT/pytest_lean.log 2>&1 || { tail -30 $OUT/pytest_lean.log; exit 1; }
tail -1 $OUT/pytest_lean.log
for r in $(seq $ROUNDS); do
  for v in 0 1; do
    for cfg in c5 c5s; do
      HD_TEAM_SWEEP_LEAN=$v timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $OUT/${cfg}_l${v}_$r.json 2> $OUT/${cfg}_l${v}_$r.err
      python -c "import json; d=json.load(open('$OUT/${cfg}_l${v}_$r.json')); p=d['path_roofline']; print('$cfg lean=$v', d['value'], d['ms_per_step'], 'layer', p['layer_ms_per_step'], 'sweep', p['sweep_ms_per_step'], 'sum', d['band_flux_sum'])"
    done
  done
done
HD_TEAM_SWEEP_LEAN=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_l1 -o kt --output-format csv -- python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-extra > $OUT/stats_l1.json 2> $OUT/stats_l1.err
python scripts/trace_timeline.py $(ls $OUT/stats_l1/kt_kernel_trace.csv $OUT/stats_l1/*/kt_kernel_trace.csv 2>/dev/null | head -1) 4 > $OUT/timeline_l1.txt
cat $OUT/timeline_l1.txt
