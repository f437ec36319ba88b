#!/bin/bash
# SQ / TCC counters of the intensity-path kernels (scripts/bench_rad.py, small shape),
# one --pmc pass per counter group:  gpurun -- bash scripts/ab/rad_pmc.sh TAG NSTR
export HD_AB=1  # the A/B switches below are read only with this opt-in
set -e -o pipefail
TAG=$1; N=${2:-16}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
RUN="python3 scripts/bench_rad.py --nstr $N --ncol 250 --steps 1 --warmup 0"
pass() {  # pass NAME COUNTERS...
  local d=$OUT/$1; shift
  echo "pmc $d: $*"
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d "$d" -o pmc --output-format csv -- $RUN > "$d.log" 2>&1
}
pass p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
pass p2 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU
pass p3 FETCH_SIZE
pass p4 WRITE_SIZE
python scripts/ab/pmc_table.py $OUT/p1 $OUT/p2 $OUT/p3 $OUT/p4 | tee $OUT/table.txt
