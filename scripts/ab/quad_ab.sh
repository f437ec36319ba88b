#!/bin/bash
# nstr 4 / 8 sweep: NN-lane teams (HD_SWEEP_QUAD=1, hd_sweep_quad_kernel) against the
# one-lane sweep.  The register-path GPU tests with the team sweep, then C1 / C3 /
# C3l alternating the two (same box), and a C3l timeline with the team sweep:
#   gpurun -- bash scripts/ab/quad_ab.sh TAG [ROUNDS]
export HD_AB=1  # the A/B switches below are read only with this opt-in
set -e -o pipefail
TAG=$1; ROUNDS=${2:-2}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
HD_SWEEP_QUAD=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_quad_sweep.py tests/test_gpu_parity.py tests/test_gpu_harp.py tests/test_gpu_band.py tests/test_gpu_physics.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_quad.log 2>&1 || { tail -30 $OUT/pytest_quad.log; exit 1; }
tail -1 $OUT/pytest_quad.log
for r in $(seq $ROUNDS); do
  for v in 0 1; do
    for cfg in c1 c3 c3l; do
      HD_SWEEP_QUAD=$v timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $OUT/${cfg}_q${v}_$r.json 2> $OUT/${cfg}_q${v}_$r.err
      python -c "import json; d=json.load(open('$OUT/${cfg}_q${v}_$r.json')); p=d.get('path_roofline', {}); print('$cfg quad=$v', d['value'], d['ms_per_step'], 'layer', p.get('layer_ms_per_step'), 'sweep', p.get('sweep_ms_per_step'), 'sum', d.get('band_flux_sum'))"
    done
  done
done
HD_SWEEP_QUAD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_q1 -o kt --output-format csv -- python3 bench.py --config c3l --steps 5 --warmup 1 --no-cpu-baseline --no-extra > $OUT/stats_q1.json 2> $OUT/stats_q1.err
python scripts/trace_timeline.py $(ls $OUT/stats_q1/kt_kernel_trace.csv $OUT/stats_q1/*/kt_kernel_trace.csv 2>/dev/null | head -1) 4 > $OUT/timeline_q1.txt
cat $OUT/timeline_q1.txt
