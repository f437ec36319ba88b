#!/bin/bash
# Team-path A/B on one box: parity of the team kernels, then C5 bench with the
# MFMA layer kernel (default) and the VALU-product one (HD_TEAM_LAYER=valu).
#   gpurun --timeout 900 -- bash scripts/gpu_team_ab.sh TAG
set -e -o pipefail
TAG=${1:-team_ab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
echo "[team_ab] $(date +%T) parity"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "vs_c_oracle or aerosol or team or graph or planck_edge or conservative" > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
echo "[team_ab] $(date +%T) c5 mfma"
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > "$OUT/c5_mfma.json" 2> "$OUT/c5_mfma.err"
cat "$OUT/c5_mfma.json"
echo "[team_ab] $(date +%T) c5 valu"
HD_TEAM_LAYER=valu timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > "$OUT/c5_valu.json" 2> "$OUT/c5_valu.err"
cat "$OUT/c5_valu.json"
