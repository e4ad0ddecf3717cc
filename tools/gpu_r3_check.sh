#!/usr/bin/env bash
# GPU tests, then the overlapped step (trace + interleaved A/B against the
# serial default) and the fused fold + scalar record (BA_REDUCE_PUB 1 / 0).
# Stops at the first fault.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited with $1 — stopping"; exit "$1" ;; esac; }
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -5 $OUT/pytest_gpu.log; stop_on_fault $rc; [ $rc = 0 ] || exit 1
fi
BA_OVERLAP=1 BA_OVERLAP_TRACE=1 timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_trace.json 2> $OUT/bench_trace.err
rc=$?; grep -A40 "overlap trace" $OUT/bench_trace.err | head -45; stop_on_fault $rc
for r in 1 2; do
  for e in "BA_OVERLAP=1" "BA_OVERLAP=0" "BA_REDUCE_PUB=0"; do
    env $e timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_ab.json 2> $OUT/bench_ab.err
    rc=$?; echo "$e $(python3 -c "import json;d=json.load(open('$OUT/bench_ab.json'));print(d['value'],d['ms_per_step'])" 2>/dev/null)"; stop_on_fault $rc
  done
done
