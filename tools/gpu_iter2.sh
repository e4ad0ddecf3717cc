#!/usr/bin/env bash
# Round-4 iteration session: the full -m gpu suite, smoke, the C3 bench, then
# the many-camera workloads (tools/gpu_big.sh: C4 full, C5 shard, profiles).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited with $1 — stopping"; exit "$1" ;; esac; }
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 1200 python3 -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread ${TESTK:+-k "$TESTK"} > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -15 $OUT/pytest_gpu.log; stop_on_fault $rc
  timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  rc=$?; tail -2 $OUT/smoke.log; stop_on_fault $rc
fi
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
rc=$?; python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('c3', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"; stop_on_fault $rc
if [ "${PROF3:-1}" = "1" ]; then
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- \
    python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_c3.json 2> $OUT/prof_c3.err
  rc=$?; stop_on_fault $rc
  echo "== c3"; python3 tools/kstats.py $OUT/prof_c3/run_kernel_stats.csv 12 | head -20
fi
bash tools/gpu_big.sh
