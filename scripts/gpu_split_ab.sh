#!/bin/bash
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/split
for f in 0 0.6 0.55 0.65 0 0.6 0.7; do
  HD_SPLIT=$f timeout -k 10 200 python bench.py --no-cpu-baseline --ngpoint 8 --steps 10 --warmup 3 > gpurun_out/split/g8_$f.json 2> gpurun_out/split/g8_$f.err
  python -c "import json; d=json.load(open('gpurun_out/split/g8_$f.json')); print('g8 split $f', d['value'], d['ms_per_step'])"
done
HD_SPLIT=0.6 timeout -k 10 200 python bench.py --ngpoint 8 --steps 5 --warmup 2 > gpurun_out/split/g8_parity.json 2> gpurun_out/split/g8_parity.err
python -c "import json; d=json.load(open('gpurun_out/split/g8_parity.json')); print('parity', d['max_rel_err_vs_cpu_restatement'], d['band_fused_vs_unfused_max_rel'])"
