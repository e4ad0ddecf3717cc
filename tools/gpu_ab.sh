#!/usr/bin/env bash
# GPU tests with the working-tree library, then the C3 bench A/B against the
# libraries given as arguments (tools/ab_bench.sh), each step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/pytest_gpu.log
  rc=$?; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 900 bash tools/ab_bench.sh "$@"
