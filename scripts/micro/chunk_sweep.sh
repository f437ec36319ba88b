# C4 at several fixed chunk sizes (0 = the automatic plan), twice, one box:
#   gpurun -- bash scripts/micro/chunk_sweep.sh
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06r
for rep in 1 2; do
for ch in 0 24576 28672 36864 40960; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra --chunk $ch > gpurun_out/r06r/c4_${ch}_${rep}.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/r06r/c4_${ch}_${rep}.json')); print('chunk $ch', d['value'], d['ms_per_step'])"
done
done
