#!/usr/bin/env bash
# Many-camera workloads on one GPU: C4 at full size (ITERATIVE_SCHUR by
# default, DENSE=1 adds DENSE_SCHUR) and the C5 shard (fp32 W), each as a
# bench line and a rocprofv3 kernel-stats run.  $AB (env variants, e.g.
# AB="BA_JR=1") repeats the two bench lines per variant.  TESTS=1 first runs
# the many-camera GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
STEPS=${STEPS:-10}
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited with $1 — stopping"; exit "$1" ;; esac; }
if [ "${TESTS:-0}" = "1" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread \
    -k "${TESTK:-c4 or c5 or 10k or many or sharded or iterative}" > $OUT/pytest_big.log 2>&1
  rc=$?; tail -8 $OUT/pytest_big.log; stop_on_fault $rc
fi
run() {  # $1 tag, rest: bench args
  local tag=$1; shift
  timeout -k 10 400 python3 -u bench.py --steps $STEPS --warmup 2 --no-cpu-baseline "$@" > $OUT/big_$tag.json 2> $OUT/big_$tag.err
  local rc=$?
  python3 -c "import json; d=json.load(open('$OUT/big_$tag.json')); print('$tag', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])" || tail -3 $OUT/big_$tag.err
  stop_on_fault $rc
}
run c4 --workload c4
run c5s --workload c5 --scale 0.125
if [ "${DENSE:-0}" = "1" ]; then run c4d --workload c4 --linear-solver dense; fi
for v in ${AB:-}; do
  ( export ${v//,/ }; run "c4_$v" --workload c4 && run "c5s_$v" --workload c5 --scale 0.125 ) || exit $?
done
if [ "${PROF:-1}" = "1" ]; then
  export TMPDIR=/tmp
  for w in "c4 --workload c4" "c5s --workload c5 --scale 0.125"; do
    set -- $w; tag=$1; shift
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$tag -o run -- \
      python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > $OUT/prof_$tag.json 2> $OUT/prof_$tag.err
    rc=$?; stop_on_fault $rc
    echo "== $tag"; python3 tools/kstats.py $OUT/prof_$tag/run_kernel_stats.csv 11 | head -26
  done
fi
exit 0
