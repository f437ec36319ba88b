#!/bin/bash
# The one GPU driver (replaces the round-1/2 one-off scripts/gpu_*.sh):
#   gpurun --timeout 1200 -- bash scripts/gpu.sh TAG STEP [STEP ...]
# Steps run in order, each under its own time limit; the first failure ends the
# call (nothing more touches the GPU after a failed step).  Outputs: gpurun_out/TAG/.
#   tests[=SEL[@K]]      pytest -m gpu in one process (SEL: comma-separated selectors,
#                        K: a -k expression with '+' for spaces)
#   abtests              pytest -m gpu scripts/ab/tests (the not-kept variants, on
#                        ab_libs/libhdisort_ab.so: build it first, scripts/ab/build_variant.sh ab)
#   smoke                __graft_entry__.smoke()
#   bench=NAME[:ARGS]    python bench.py ARGS              > bench_NAME.json
#   stats=NAME[:ARGS]    rocprofv3 --kernel-trace --stats of bench.py ARGS:
#                        stats_NAME/ (kernel_stats.csv, kernel_trace.csv) + bench line
#   pmc=NAME[:NSTR]      FETCH_SIZE and WRITE_SIZE passes (one --pmc pass each) over
#                        scripts/pmc_run.py (one chunk of the C4 / C5 shape)
#   sq=NAME[:NSTR]       SQ instruction-mix / MFMA / LDS passes over scripts/pmc_run.py
#   rad=NAME[:ARGS]      python scripts/bench_rad.py ARGS  > rad_NAME.json
#   radstats=NAME[:ARGS] rocprofv3 --kernel-trace --stats of scripts/bench_rad.py ARGS
#   radsq=NAME[:ARGS]    SQ / FETCH_SIZE passes (one --pmc pass each) over one bench_rad.py step
# ARGS are comma-separated (bench=c5:--config,c5,--steps,5).
set -e -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
say() { echo "[gpu] $(date +%T) $*"; }
args_of() { echo "${1//,/ }"; }

pmc_pass() {  # pmc_pass DIR NSTR COUNTERS...
  local d=$1 nstr=$2; shift 2
  say "pmc $d: $*"
  PMC_NSTR=$nstr timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d "$d" -o pmc \
    --output-format csv -- python3 scripts/pmc_run.py > "$d.log" 2>&1
}

for step in "$@"; do
  kind=${step%%=*}
  val=${step#*=}
  [ "$val" = "$step" ] && val=""
  name=${val%%:*}
  rest=${val#*:}
  [ "$rest" = "$val" ] && rest=""
  case $kind in
    tests)
      v=${val:-tests}
      sel=$(args_of "${v%%@*}")
      kexpr=""
      [ "${v#*@}" != "$v" ] && kexpr=${v#*@} && kexpr=${kexpr//+/ }
      say "pytest -m gpu $sel ${kexpr:+-k \"$kexpr\"}"
      HD_MARGINS_OUT=$OUT/parity_margins.json timeout -k 10 840 python -u -m pytest $sel -m gpu ${kexpr:+-k "$kexpr"} -x -v --timeout 120 \
        --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
      tail -3 "$OUT/pytest_gpu.log" ;;
    abtests)
      say "pytest -m gpu scripts/ab/tests"
      timeout -k 10 600 python -u -m pytest scripts/ab/tests -m gpu -x -v --timeout 300 \
        --timeout-method thread > "$OUT/pytest_ab.log" 2>&1 || { tail -40 "$OUT/pytest_ab.log"; exit 1; }
      tail -3 "$OUT/pytest_ab.log" ;;
    smoke)
      say smoke
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
        || { cat "$OUT/smoke.log"; exit 1; }
      tail -2 "$OUT/smoke.log" ;;
    bench)
      say "bench $name: $(args_of "$rest")"
      timeout -k 10 420 python bench.py $(args_of "$rest") > "$OUT/bench_$name.json" \
        2> "$OUT/bench_$name.err" || { tail -20 "$OUT/bench_$name.err"; exit 1; }
      cat "$OUT/bench_$name.json" ;;
    stats)
      say "rocprofv3 --kernel-trace --stats bench.py $(args_of "$rest")"
      timeout -k 10 480 rocprofv3 --kernel-trace --stats -d "$OUT/stats_$name" -o kt \
        --output-format csv -- python3 bench.py $(args_of "$rest") > "$OUT/stats_$name.json" \
        2> "$OUT/stats_$name.err" || { tail -20 "$OUT/stats_$name.err"; exit 1; }
      cat "$OUT/stats_$name.json" ;;
    pmc)
      pmc_pass "$OUT/pmc_${name}_fetch" "${rest:-16}" FETCH_SIZE
      pmc_pass "$OUT/pmc_${name}_write" "${rest:-16}" WRITE_SIZE ;;
    sq)
      n=${rest:-16}
      pmc_pass "$OUT/sq_${name}_p1" "$n" SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
        SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
      pmc_pass "$OUT/sq_${name}_p2" "$n" SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 \
        SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
        SQ_INSTS_VMEM_WR SQ_INSTS_SALU
      pmc_pass "$OUT/sq_${name}_p3" "$n" SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES \
        SQ_INSTS_VALU_MFMA_F64 SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM \
        SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC ;;
    rad)
      say "bench_rad $name: $(args_of "$rest")"
      timeout -k 10 420 python scripts/bench_rad.py $(args_of "$rest") > "$OUT/rad_$name.json" \
        2> "$OUT/rad_$name.err" || { tail -20 "$OUT/rad_$name.err"; exit 1; }
      cat "$OUT/rad_$name.json" ;;
    radstats)
      say "rocprofv3 --kernel-trace --stats bench_rad.py $(args_of "$rest")"
      timeout -k 10 480 rocprofv3 --kernel-trace --stats -d "$OUT/radstats_$name" -o kt \
        --output-format csv -- python3 scripts/bench_rad.py $(args_of "$rest") \
        > "$OUT/radstats_$name.json" 2> "$OUT/radstats_$name.err" || { tail -20 "$OUT/radstats_$name.err"; exit 1; }
      cat "$OUT/radstats_$name.json" ;;
    radsq)
      for p in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
               "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64" \
               "FETCH_SIZE"; do
        d="$OUT/radsq_${name}_$(echo $p | cut -d' ' -f1)"
        say "pmc $d: $p"
        timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $p -d "$d" -o pmc --output-format csv \
          -- python3 scripts/bench_rad.py --steps 1 --warmup 0 $(args_of "$rest") > "$d.log" 2>&1
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
say done
