#!/bin/bash
# SQ instruction-mix / stall counters for the intensity path's kernels (scripts/bench_rad.py, one step)
set -e -o pipefail
OUT=gpurun_out/${1:-sq_rad}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d "$OUT/p1" -o pmc --output-format csv -- python3 scripts/bench_rad.py --steps 1 --warmup 0 > "$OUT/p1.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU -d "$OUT/p2" -o pmc --output-format csv -- python3 scripts/bench_rad.py --steps 1 --warmup 0 > "$OUT/p2.log" 2>&1 || echo "p2 failed"
echo done
