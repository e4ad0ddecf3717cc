#!/usr/bin/env bash
# Instruction-cache check of the persistent Cholesky: the FULL (unrolled
# sub-panel) build against the general form (BA_CHOL_PERSIST_GENERAL, 60 vs
# 80 KB of code): timing, then SQC_ICACHE_* / SQ_IFETCH counters per build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited with $1 — stopping"; exit "$1" ;; esac; }
for b in chol_bench_ns chol_bench_gen; do
  for n in 1194 1152; do
    timeout -k 5 120 tools/$b $n > $OUT/e_${b}_$n.txt 2>&1; rc=$?
    echo "== $b $n"; grep -E "persistent factor|differing|residual" $OUT/e_${b}_$n.txt | head -8; stop_on_fault $rc
  done
done
for b in chol_bench_ns chol_bench_gen; do
  timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES -d $OUT/pmc_ic_$b -o ic \
    --output-format csv -- tools/$b 1194 > $OUT/pmc_ic_$b.log 2>&1; rc=$?; echo "pmc ic $b rc=$rc"; stop_on_fault $rc
  timeout -s KILL 60 rocprofv3 --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/pmc_if_$b -o if \
    --output-format csv -- tools/$b 1194 > $OUT/pmc_if_$b.log 2>&1; rc=$?; echo "pmc if $b rc=$rc"; stop_on_fault $rc
done
find $OUT/pmc_ic_* $OUT/pmc_if_* -name "*counter_collection.csv" | head
