#!/usr/bin/env bash
# GPU suite + smoke after the ACC point-step prefetch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/v
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/v/gpu_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/v/gpu_tests.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v/smoke.txt 2>&1
rc=$?; tail -1 gpurun_out/v/smoke.txt; exit $rc
