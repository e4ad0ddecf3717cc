#!/usr/bin/env bash
# rocprofv3 kernel stats of the C3 bench per BA_OVERLAP mode (0 serial, 2
# serialised signalled pair pass + row-waiting factorisation, 1 overlapped)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited with $1 — stopping"; exit "$1" ;; esac; }
for ov in ${MODES:-0 2 1}; do
  BA_OVERLAP=$ov timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_ov$ov -o run -- \
    python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_ov$ov.json 2> $OUT/prof_ov$ov.err
  rc=$?; stop_on_fault $rc
  echo "== BA_OVERLAP=$ov $(python3 -c "import json;d=json.load(open('$OUT/prof_ov$ov.json'));print(d['value'],d['ms_per_step'])" 2>/dev/null)"
  python3 tools/kstats.py $OUT/prof_ov$ov/run_kernel_stats.csv 2>/dev/null | grep -v stream_copy | head -${TOP:-6} || true
  python3 tools/ktimeline.py $OUT/prof_ov$ov/run_kernel_trace.csv 2>/dev/null || true
done
