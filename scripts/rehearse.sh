#!/bin/bash
# One-GPU rehearsal of bench.py's N-rank path (HD_BENCH_REHEARSE=1: the ranks share
# the box's GPU and all-reduce over gloo), N = 1, 2, 4, 8, for C4 and C5.  The
# band_flux_sum checksum of every line must equal the N = 1 line's to all printed
# digits (the g-point shards' partial band sums, completed by the all-reduce).
#   gpurun -- bash scripts/rehearse.sh TAG [CONFIG ...]
set -e -o pipefail
TAG=${1:?tag}; shift
CONFIGS=${*:-c4 c5}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in $CONFIGS; do
  for n in 1 2 4 8; do
    echo "[rehearse] $(date +%T) $c N=$n"
    HD_BENCH_REHEARSE=1 timeout -k 10 400 python bench.py --gpus $n --config $c --steps 3 --warmup 1 \
      --no-extra --no-cpu-baseline > $OUT/rehearse_${c}_n$n.json 2> $OUT/rehearse_${c}_n$n.err \
      || { tail -20 $OUT/rehearse_${c}_n$n.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/rehearse_${c}_n$n.json')); print('$c N=$n', d['n_gpus'], d['value'], d['ms_per_step'], 'band_flux_sum', repr(d['band_flux_sum']))"
  done
done
