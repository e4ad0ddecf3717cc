#!/usr/bin/env bash
# Iteration GPU session: full -m gpu suite, smoke, C3 bench (+ A/B env
# variants given in $AB, e.g. AB="BA_JR=1 BA_CHOL_PERSIST=0"), rocprofv3 stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited with $1 — stopping"; exit "$1" ;; esac; }
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 1200 python3 -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -15 $OUT/pytest_gpu.log; stop_on_fault $rc
  timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  rc=$?; tail -2 $OUT/smoke.log; stop_on_fault $rc
fi
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; stop_on_fault $rc
for v in ${AB:-}; do
  timeout -k 10 300 env ${v//,/ } python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_$v.json 2>> $OUT/bench.err
  rc=$?; echo "== $v"; python3 -c "import json,sys; d=json.load(open('$OUT/bench_$v.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"; stop_on_fault $rc
done
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench2.json 2>> $OUT/bench.err
rc=$?; python3 -c "import json; d=json.load(open('$OUT/bench2.json')); print('repeat', d['value'], d['ms_per_step'])"; stop_on_fault $rc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err
rc=$?; stop_on_fault $rc
python3 tools/kstats.py $OUT/prof/run_kernel_stats.csv 11 | head -24
