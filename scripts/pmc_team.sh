#!/bin/bash
# Counters of the team kernels (nstr 18..32) on one C5-shaped chunk (PMC_NSTR=32:
# 16 384 solves, scripts/pmc_run.py): SQ instruction mix (two passes), MFMA, and
# HBM bytes (FETCH_SIZE, WRITE_SIZE in passes of their own).
#   gpurun -- bash scripts/pmc_team.sh TAG
set -e -o pipefail
OUT=gpurun_out/${1:-pmc_team}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PMC_NSTR=${PMC_NSTR:-32}
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
pass() {  # pass NAME COUNTERS...
  local n=$1; shift
  echo "[pmc] $(date +%T) $n: $*"
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$n" -o pmc --output-format csv -- python3 scripts/pmc_run.py > "$OUT/$n.log" 2>&1
}
pass p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
pass p2 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU
pass p3 SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC
pass pmc_fetch FETCH_SIZE
pass pmc_write WRITE_SIZE
echo "[pmc] $(date +%T) done"
