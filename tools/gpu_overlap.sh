#!/usr/bin/env bash
# Overlapped DENSE_SCHUR step on one GPU box: the GPU tests, C3 bench with the
# overlap on / off (interleaved), a rocprofv3 kernel trace of the default.
# A fault / abort / timeout stops the script (no further GPU work).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited with $1 — stopping"; exit "$1" ;; esac; }
if [ "${TESTS:-1}" = "1" ]; then
  echo "== pytest -m gpu"
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -15 $OUT/pytest_gpu.log; stop_on_fault $rc
  [ $rc = 0 ] || exit 1
fi
echo "== bench A/B (BA_OVERLAP 1 / 0, interleaved)"
for r in 1 2; do
  for ov in 1 0; do
    BA_OVERLAP=$ov timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_ov$ov.json 2> $OUT/bench_ov$ov.err
    rc=$?; echo "overlap=$ov $(python3 -c "import json;d=json.load(open('$OUT/bench_ov$ov.json'));print(d['value'],d['ms_per_step'])" 2>/dev/null)"; stop_on_fault $rc
  done
done
echo "== rocprofv3 kernel trace (default)"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err
rc=$?; stop_on_fault $rc
python3 tools/kstats.py $OUT/prof/run_kernel_stats.csv 2>/dev/null | head -25 || true
