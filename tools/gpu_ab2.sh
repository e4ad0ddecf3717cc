#!/usr/bin/env bash
# GPU tests with an alternative library build ($1), then the C3 bench A/B of the
# in-tree library against it (tools/ab_bench.sh); each step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
BA_HIP_LIB="$1" timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider 2>&1 | tee gpurun_out/pytest_gpu_alt.log
rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/ab_bench.sh "$1"
