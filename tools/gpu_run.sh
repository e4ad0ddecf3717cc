#!/usr/bin/env bash
# One parameterised GPU-box run (replaces the per-experiment gpu_*.sh scripts
# of rounds 1-5).  Usage, from the repo root on the box:
#
#   tools/gpu_run.sh OUTDIR STEP [STEP ...]
#
# Each STEP is one shell word; fields are ':'-separated, and '+' stands for a
# space inside bench / pytest arguments:
#   tests[:EXPR]               pytest -m gpu [-k EXPR] (e.g. tests:blocks+or+persistent)
#   smoke                      __graft_entry__.smoke()
#   bench:TAG[:ARGS]           python bench.py ARGS > OUTDIR/bench_TAG.json
#   prof:TAG[:ARGS]            rocprofv3 --kernel-trace --stats of bench.py ARGS
#                              (summary: OUTDIR/prof_TAG/.../kernel_stats.csv)
#   hbm:TAG[:ARGS]             FETCH_SIZE and WRITE_SIZE passes (separate, as the
#                              guide prescribes), summarised by tools/pmc_summary.py
#   sq:TAG[:ARGS]              one SQ / LDS counter pass, tools/pmc_table.py
#   chol:N[:BIN[:TAG]]         tools/chol_bench_ns (or BIN) at order N (output file tagged TAG)
#   env:VAR=VALUE              exported for the following steps
#   unset:VAR                  unexported
# Every GPU step has its own time limit; a step that faults, aborts or times
# out ends the run (exit 0/1 from a step is recorded and the run goes on).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:?outdir}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
T_BENCH=${T_BENCH:-600}
SQSET="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU"
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited with $1 — stopping"; exit "$1" ;; esac; }
show() {
  python3 -c 'import json,sys
try:
    d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
except Exception as e:
    print(sys.argv[2], "no json:", e); sys.exit(0)
t = d.get("trajectory") or {}; c = d.get("cpu_baseline") or {}
print(sys.argv[2], d.get("value"), "M-obs/s", d.get("ms_per_step"), "ms median", d.get("ms_per_step_median"),
      "roofline", (d.get("roofline") or {}).get("frac"), "cpu", c.get("value"), "cg", t.get("linear_solver_iterations"))' "$1" "$2" || true
}
for step in "$@"; do
  IFS=: read -r kind a1 a2 a3 <<< "$step"
  a1=${a1:-}; a2=${a2:-}; a3=${a3:-}
  echo "== $step"
  case $kind in
    env) export "$a1"; continue ;;
    unset) unset "$a1"; continue ;;
    tests)
      kexpr=(); [ -n "$a1" ] && kexpr=(-k "${a1//+/ }")
      timeout -k 10 1100 python3 -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread "${kexpr[@]}" \
        > "$OUT/pytest_gpu.log" 2>&1
      rc=$?; tail -6 "$OUT/pytest_gpu.log" ;;
    smoke)
      timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      rc=$?; tail -1 "$OUT/smoke.log" ;;
    bench)
      timeout -k 10 $T_BENCH python3 -u bench.py ${a2//+/ } > "$OUT/bench_$a1.json" 2> "$OUT/bench_$a1.err"
      rc=$?; show "$OUT/bench_$a1.json" "$a1" ;;
    prof)
      timeout -k 10 $T_BENCH rocprofv3 --kernel-trace --stats -d "$OUT/prof_$a1" -o run --output-format csv -- \
        python3 -u bench.py --no-cpu-baseline ${a2//+/ } > "$OUT/prof_$a1.json" 2> "$OUT/prof_$a1.err"
      rc=$?; show "$OUT/prof_$a1.json" "prof_$a1"
      f=$(find "$OUT/prof_$a1" -name '*kernel_stats.csv' | head -1)
      [ -n "$f" ] && { python3 tools/kstats.py "$f" > "$OUT/prof_$a1.txt" 2>&1; head -16 "$OUT/prof_$a1.txt"; } ;;
    hbm)
      rc=0
      for ctr in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmc_${a1}_$ctr" -o run -- \
          python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline ${a2//+/ } > "$OUT/pmc_${a1}_$ctr.json" 2> "$OUT/pmc_${a1}_$ctr.err"
        r=$?; echo "$a1 $ctr rc=$r"; [ $r -gt $rc ] && rc=$r
        case $r in 0|1) ;; *) break ;; esac
      done
      python3 tools/pmc_summary.py "$OUT/pmc_${a1}_FETCH_SIZE" "$OUT/pmc_${a1}_WRITE_SIZE" "$OUT/pmc_$a1.json" \
        > "$OUT/pmc_${a1}_hbm.txt" 2>&1 || true
      head -20 "$OUT/pmc_${a1}_hbm.txt" ;;
    sq)
      timeout -s KILL 300 rocprofv3 --pmc $SQSET --output-format csv -d "$OUT/pmc_${a1}_SQ" -o run -- \
        python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline ${a2//+/ } > "$OUT/pmc_${a1}_SQ.json" 2> "$OUT/pmc_${a1}_SQ.err"
      rc=$?
      python3 tools/pmc_table.py "$OUT/pmc_${a1}_SQ" > "$OUT/pmc_${a1}_sq.txt" 2>&1 || true
      head -20 "$OUT/pmc_${a1}_sq.txt" ;;
    chol)
      bin=${a2:-tools/chol_bench_ns}
      cf="$OUT/chol_$(basename "$bin")_$a1${a3:+_$a3}.txt"
      timeout -k 5 180 "$bin" "$a1" > "$cf" 2>&1
      rc=$?; grep -E "factor (flow|streamed)|differing|residual" "$cf" | tail -5 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "$step rc=$rc"
  stop_on_fault $rc
done
exit 0
