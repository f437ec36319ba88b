#!/bin/bash
# Pipeline change check: register-path parity/band/concurrency tests, bench lines
# (C4, the 8/4-GPU rank shapes, C4+Planck) and a kernel timeline of C4.
#   gpurun --timeout 900 -- bash scripts/gpu_pipe_check.sh TAG
set -e -o pipefail
TAG=${1:-pipe}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_band.py tests/test_gpu_concurrency.py tests/test_gpu_distributed.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for cfg in "c4a:" "g8a:--ngpoint 8" "g16:--ngpoint 16" "c4b:" "g8b:--ngpoint 8" "c4p:--planck"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 $args > "$OUT/$name.json" 2> "$OUT/$name.err"
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['ms_per_step'], 'layer', d['roofline']['avg_launch_ms'])"
done
timeout -k 10 180 rocprofv3 --kernel-trace -d "$OUT/raw" -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err"
cp "$(find "$OUT/raw" -name '*kernel_trace.csv' | head -1)" "$OUT/kernel_trace.csv"
echo done
