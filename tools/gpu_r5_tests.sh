#!/usr/bin/env bash
# The full -m gpu suite and smoke at the working tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -6 $OUT/pytest_gpu.log
case $rc in 0|1) ;; *) echo "pytest exited $rc — stopping"; exit $rc ;; esac
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc2=$?; tail -2 $OUT/smoke.log
exit $(( rc > rc2 ? rc : rc2 ))
