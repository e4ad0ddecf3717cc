#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 5 120 tools/chol_bench 1194 > gpurun_out/l_chol_bench_1194.txt 2>&1; rc=$?
grep -E "persistent|critical|sub-panel 3|tail|differing" gpurun_out/l_chol_bench_1194.txt | head -20
exit $rc
