#!/usr/bin/env bash
# Overlapped DENSE_SCHUR step, quick check: its bitwise test, one traced C3
# bench (BA_OVERLAP_TRACE=1 prints one step's timeline), then an interleaved
# A/B of BA_OVERLAP=1 against the serial default.  Stops at the first fault.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited with $1 — stopping"; exit "$1" ;; esac; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k overlapped -x -q --timeout 120 --timeout-method thread > $OUT/pytest_ov.log 2>&1
rc=$?; tail -5 $OUT/pytest_ov.log; stop_on_fault $rc; [ $rc = 0 ] || exit 1
BA_OVERLAP=1 BA_OVERLAP_TRACE=1 timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_trace.json 2> $OUT/bench_trace.err
rc=$?; grep -A40 "overlap trace" $OUT/bench_trace.err | head -45; stop_on_fault $rc
for r in 1 2; do
  for ov in 1 0; do
    BA_OVERLAP=$ov timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_ov$ov.json 2> $OUT/bench_ov$ov.err
    rc=$?; echo "overlap=$ov $(python3 -c "import json;d=json.load(open('$OUT/bench_ov$ov.json'));print(d['value'],d['ms_per_step'])" 2>/dev/null)"; stop_on_fault $rc
  done
done
