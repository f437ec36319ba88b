#!/bin/bash
# nstr 18..32 user angles: team/MFMA kernel pair against the rolled one-lane kernel
# (HD_RAD_USER=rolled).  Radiance GPU tests, then scripts/bench_rad.py A/B and a
# kernel-stats profile of the team version:
#   gpurun -- bash scripts/ab/rad_user_ab.sh TAG
export HD_AB=1  # the A/B switches below are read only with this opt-in
set -e -o pipefail
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_radiance.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_rad.log 2>&1 || { tail -40 $OUT/pytest_rad.log; exit 1; }
tail -2 $OUT/pytest_rad.log
for n in 32 24; do
  timeout -k 10 300 python scripts/bench_rad.py --nstr $n --steps 3 --warmup 1 > $OUT/rad_n${n}_team.json
  cat $OUT/rad_n${n}_team.json
done
timeout -k 10 300 python scripts/bench_rad.py --nstr 16 --steps 5 --warmup 2 > $OUT/rad_n16.json
cat $OUT/rad_n16.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_n32 -o kt --output-format csv -- python3 scripts/bench_rad.py --nstr 32 --steps 2 --warmup 1 > $OUT/stats_n32.json
cut -d, -f1-5 $(ls $OUT/stats_n32/kt_kernel_stats.csv $OUT/stats_n32/*/kt_kernel_stats.csv 2>/dev/null | head -1) | head -12
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_n16 -o kt --output-format csv -- python3 scripts/bench_rad.py --nstr 16 --steps 3 --warmup 1 > $OUT/stats_n16.json
cut -d, -f1-5 $(ls $OUT/stats_n16/kt_kernel_stats.csv $OUT/stats_n16/*/kt_kernel_stats.csv 2>/dev/null | head -1) | head -12
