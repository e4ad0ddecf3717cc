#!/usr/bin/env bash
# Interleaved A/B of env variants on the C3 bench (one box, ROUNDS rounds),
# then a rocprofv3 kernel-stats run per variant.  $AB: space-separated
# variants, each a comma-separated env list ("-" = defaults), e.g.
# AB="- BA_PAIRS_DMA=1".  TESTK: a -m gpu test selection run first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited with $1 — stopping"; exit "$1" ;; esac; }
if [ -n "${TESTK:-}" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread -k "$TESTK" > $OUT/pytest_ab.log 2>&1
  rc=$?; tail -5 $OUT/pytest_ab.log; stop_on_fault $rc
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${AB:--}; do
    tag=${v//,/_}
    ( [ "$v" != "-" ] && export ${v//,/ }
      timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/ab_$tag.json 2> $OUT/ab_$tag.err
      rc=$?
      python3 -c "import json; d=json.load(open('$OUT/ab_$tag.json')); print('r$r', '$v', d['value'], d['ms_per_step'], d.get('ms_per_step_median'))" || tail -3 $OUT/ab_$tag.err
      exit $rc ) || stop_on_fault $?
  done
done
if [ "${PROF:-1}" = "1" ]; then
  export TMPDIR=/tmp
  for v in ${AB:--}; do
    tag=${v//,/_}
    ( [ "$v" != "-" ] && export ${v//,/ }
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_ab_$tag -o run -- \
        python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/prof_ab_$tag.json 2> $OUT/prof_ab_$tag.err
      rc=$?
      echo "== $v"; python3 tools/kstats.py $OUT/prof_ab_$tag/run_kernel_stats.csv 12 | head -${KTOP:-8}
      exit $rc ) || stop_on_fault $?
  done
fi
exit 0
