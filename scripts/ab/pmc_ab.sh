#!/bin/bash
# SQ stall counters + I-cache counters for library variants mb/<name> (one C4 chunk)
export HD_AB=1  # the A/B switches below are read only with this opt-in
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmcab; mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
for v in "$@"; do
  export HD_LIB_PATH=$PWD/mb/$v/libhdisort.so
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d "$OUT/$v.p1" -o pmc --output-format csv -- python3 scripts/pmc_run.py > "$OUT/$v.p1.log" 2>&1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS -d "$OUT/$v.p2" -o pmc --output-format csv -- python3 scripts/pmc_run.py > "$OUT/$v.p2.log" 2>&1 || echo "$v p2 failed"
done
grep -h "SQC_ICACHE\|SQ_INST_LEVEL\|SQ_IFETCH\|SQ_INSTS_\|LDS_BANK" $OUT/counters.txt | head -40 > $OUT/counters_sel.txt || true
echo done
