#!/bin/bash
# End-of-round verification on one box: every GPU test, the smoke, the driver's bench
# line, C5 / C1 lines, radiance throughput at nstr 32 / 24 / 16 and a kernel-stats
# profile of the nstr-32 radiance run.  gpurun -- bash scripts/ab/final_r04.sh TAG
export HD_AB=1  # the A/B switches below are read only with this opt-in
set -e -o pipefail
TAG=$1
bash scripts/gpu.sh $TAG tests smoke bench=c4 "bench=c5:--config,c5,--steps,10,--warmup,3,--no-extra" \
  "bench=c1:--config,c1,--steps,50,--warmup,5,--no-extra" \
  "rad=n32:--nstr,32,--steps,3,--warmup,1" "rad=n24:--nstr,24,--steps,3,--warmup,1" \
  "rad=n16:--nstr,16,--steps,5,--warmup,2" \
  "radstats=n32:--nstr,32,--steps,2,--warmup,1"
