export HD_AB=1  # the A/B switches below are read only with this opt-in
set -e -o pipefail
mkdir -p gpurun_out/gab
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
for g in "" "--graph"; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $g > gpurun_out/gab/c4_${rep}${g}.json 2> gpurun_out/gab/c4_${rep}${g}.err
  python -c "import json; d=json.load(open('gpurun_out/gab/c4_${rep}${g}.json')); print('c4 $g', d['value'], d['ms_per_step'])"
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --ngpoint 8 $g > gpurun_out/gab/g8_${rep}${g}.json 2> gpurun_out/gab/g8_${rep}${g}.err
  python -c "import json; d=json.load(open('gpurun_out/gab/g8_${rep}${g}.json')); print('g8 $g', d['value'], d['ms_per_step'])"
done
done
