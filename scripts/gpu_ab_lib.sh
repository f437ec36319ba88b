#!/bin/bash
# A/B of library variants (mb/NAME/libhdisort.so via HD_LIB_PATH) on one box:
# the in-tree library first, then each variant, same bench arguments.
#   gpurun --timeout 900 -- bash scripts/gpu_ab_lib.sh TAG "BENCH ARGS" NAME...
set -e -o pipefail
TAG=$1; ARGS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[ab] $(date +%T) in-tree: $ARGS"
timeout -k 10 300 python bench.py --no-cpu-baseline $ARGS > "$OUT/tree.json" 2> "$OUT/tree.err"
python -c "import json;d=json.load(open('$OUT/tree.json'));print('tree', d['value'], d['roofline']['avg_launch_ms'])"
for n in "$@"; do
  echo "[ab] $(date +%T) $n"
  HD_LIB_PATH=$GRAFT_REPO_ROOT/mb/$n/libhdisort.so timeout -k 10 300 python bench.py --no-cpu-baseline $ARGS > "$OUT/$n.json" 2> "$OUT/$n.err"
  python -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', d['value'], d['roofline']['avg_launch_ms'])"
done
