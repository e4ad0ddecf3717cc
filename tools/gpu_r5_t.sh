#!/usr/bin/env bash
# The camera pass on a side stream: GPU suite, then C3 and C4 (fixed radius)
# A/B against the single-stream build (CAM_SIDE_STREAM=0), and C3 kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/t
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/t/gpu_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/t/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 tools/ab_bench.sh bundleadjustment_amd/ab/libba_noside.so || exit 1
BENCH_ARGS="--workload c4 --mode fixed" timeout -k 10 900 tools/ab_bench.sh bundleadjustment_amd/ab/libba_noside.so || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/t/prof_c3 -o run --output-format csv -- \
  python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/t/prof_c3.json 2>&1
echo "prof rc=$?"
