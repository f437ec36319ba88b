#!/bin/bash
# Fused register path: parity (fused vs pipeline bitwise, oracle subsample, band tests),
# then bench lines (C4 fused; the 8/4/2-GPU rank shapes) and a C4 kernel timeline.
#   gpurun --timeout 900 -- bash scripts/gpu_fused_check.sh TAG
set -e -o pipefail
TAG=${1:-fused}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fused or headline or chunk" -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for cfg in "c4:" "g32:--ngpoint 32" "c4b:" "c4p:--planck"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 $args > "$OUT/$name.json" 2> "$OUT/$name.err"
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['ms_per_step'], 'maxrel', d.get('max_rel_err_vs_cpu', d.get('parity')))"
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/raw" -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err"
cp "$(find "$OUT/raw" -name '*kernel_trace.csv' | head -1)" "$OUT/kernel_trace.csv"
cp "$(find "$OUT/raw" -name '*kernel_stats.csv' | head -1)" "$OUT/kernel_stats.csv"
echo done
