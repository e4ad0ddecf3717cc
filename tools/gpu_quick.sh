#!/usr/bin/env bash
# Quick GPU iteration: parity tests, bench (no CPU baseline), rocprofv3 kernel stats.
# Each GPU step has its own time limit; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -15 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; tail -3 $OUT/bench.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/prof_bench.json 2> $OUT/prof.err
rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/prof.err; exit $rc; }
python3 tools/kstats.py $OUT/prof/run_kernel_stats.csv | head -25
