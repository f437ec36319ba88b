#!/bin/bash
# Parity tests + C4/C5 bench lines + one FETCH_SIZE pass of a C4 chunk (A/B of a kernel change).
#   gpurun --timeout 900 -- bash scripts/gpu_ab_quick.sh TAG
set -e -o pipefail
TAG=${1:-ab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_band.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err"
timeout -k 10 300 python bench.py --no-cpu-baseline --config c5 --steps 3 --warmup 1 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err"
timeout -k 10 300 python bench.py --no-cpu-baseline --ngpoint 8 > "$OUT/bench_g8.json" 2> "$OUT/bench_g8.err"
python - "$OUT" <<'PY'
import json, sys
for c in ("c4", "c5", "g8"):
    d = json.load(open(f"{sys.argv[1]}/bench_{c}.json"))
    print(c, d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["path_roofline"]["frac"])
PY
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o pmc --output-format csv -- \
    python3 scripts/pmc_run.py > "$OUT/pmc_fetch.log" 2>&1
echo done
