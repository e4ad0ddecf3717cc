#!/usr/bin/env bash
# Diagonal slices in the pair pass's launch: GPU suite, then C3 A/B against
# the separate diagonal launch (DIAG_IN_PAIRS=0 build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/r/gpu_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r/gpu_tests.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 tools/ab_bench.sh bundleadjustment_amd/ab/libba_nodiag.so || exit 1
timeout -k 10 600 tools/ab_bench.sh bundleadjustment_amd/ab/libba_nodiag.so || exit 1
