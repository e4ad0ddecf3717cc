#!/usr/bin/env bash
# Column-ordered overlapped step: the pair pass's grid cap (BA_PAIRS_GRID)
# sets how many block columns are in flight at once, i.e. how strictly the
# columns complete in order.  One traced run per cap, then an interleaved A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited with $1 — stopping"; exit "$1" ;; esac; }
for g in ${GRIDS:-256 512}; do
  echo "== grid cap $g"
  BA_PAIRS_GRID=$g BA_OVERLAP=1 BA_OVERLAP_TRACE=1 timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_trace_$g.json 2> $OUT/bench_trace_$g.err
  rc=$?; grep -A21 "overlap trace" $OUT/bench_trace_$g.err | head -22; stop_on_fault $rc
done
for r in 1 2; do
  for e in ${AB:-"BA_OVERLAP=0" "BA_OVERLAP=1 BA_PAIRS_GRID=256" "BA_OVERLAP=1 BA_PAIRS_GRID=512"}; do
    env $e timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_ab.json 2> $OUT/bench_ab.err
    rc=$?; echo "$e $(python3 -c "import json;d=json.load(open('$OUT/bench_ab.json'));print(d['value'],d['ms_per_step'])" 2>/dev/null)"; stop_on_fault $rc
  done
done
