#!/usr/bin/env bash
# MIXED_FP32 back substitution from the accumulated CG products: the mixed /
# pacc GPU tests, then C5-shard A/B against the previous build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/n
timeout -k 10 600 python3 -u -m pytest tests/test_pcg.py -m gpu -q -rf --timeout 200 --timeout-method thread \
  -k "accumulated or mixed" > gpurun_out/n/tests.txt 2>&1
rc=$?; tail -3 gpurun_out/n/tests.txt; [ $rc -le 1 ] || exit $rc
BENCH_ARGS="--workload c5 --scale 0.125 --mode fixed" timeout -k 10 600 tools/ab_bench.sh bundleadjustment_amd/ab/libba_head.so
