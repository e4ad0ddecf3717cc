#!/usr/bin/env bash
# Cholesky-focused GPU session: chol_bench (per-step vs persistent, stamps),
# the dense parity tests, a C3 bench and its rocprofv3 kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited with $1 — stopping"; exit "$1" ;; esac; }
for n in 1194 600; do
  timeout -k 10 120 tools/chol_bench $n > $OUT/chol_bench_$n.txt 2>&1
  rc=$?; grep -E "persistent|factor total|residual" $OUT/chol_bench_$n.txt; stop_on_fault $rc
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -x --timeout 300 \
  --timeout-method thread -k "persistent or solve_matches or c3_first or c4_shard_first" > $OUT/pytest_chol.log 2>&1
rc=$?; tail -3 $OUT/pytest_chol.log; stop_on_fault $rc
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; stop_on_fault $rc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err
rc=$?; stop_on_fault $rc
python3 tools/kstats.py $OUT/prof/run_kernel_stats.csv 2>/dev/null | head -25 || true
