#!/usr/bin/env bash
# The GPU tests, then an interleaved A/B (tools/gpu_ab_prof.sh; AB as there).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -6 gpurun_out/pytest_gpu.log
  [ $rc = 0 ] || exit $rc
fi
bash tools/gpu_ab_prof.sh
