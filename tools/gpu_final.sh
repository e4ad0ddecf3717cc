#!/usr/bin/env bash
# Round-end validation on one GPU: the full -m gpu suite, smoke, the default
# bench line (C3, with the CPU baseline), C3 kernel stats, C3 HBM PMC passes
# (profiles/pmc_c3.json feeds roofline.traffic), then C4 full size and the C5
# shard with their kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited with $1 — stopping"; exit "$1" ;; esac; }
timeout -k 10 1200 python3 -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -4 $OUT/pytest_gpu.log; stop_on_fault $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -2 $OUT/smoke.log; stop_on_fault $rc
timeout -k 10 600 python3 -u bench.py > $OUT/final_bench.json 2> $OUT/final_bench.err
rc=$?; python3 -c "import json; d=json.load(open('$OUT/final_bench.json')); print('c3', d['value'], d['ms_per_step'], d.get('ms_per_step_median'), d['roofline']['frac'], d['cpu_baseline']['value'])"; stop_on_fault $rc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- \
  python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_c3.json 2> $OUT/prof_c3.err
rc=$?; stop_on_fault $rc
echo "== c3"; python3 tools/kstats.py $OUT/prof_c3/run_kernel_stats.csv 12 | head -16
WL="c3" bash tools/gpu_pmc4.sh || exit $?
TESTS=0 bash tools/gpu_big.sh
