#!/usr/bin/env bash
# Many-camera check: the C4-shard bench, then C4 full size and the C5 shard
# with their kernel stats (tools/gpu_big.sh), and the C3 bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
AB="-" ROUNDS=1 KTOP=12 BENCH_ARGS="--workload c4 --scale 0.125" bash tools/gpu_ab_c3.sh || exit $?
TESTS=0 bash tools/gpu_big.sh || exit $?
AB="-" ROUNDS=2 PROF=0 bash tools/gpu_ab_c3.sh
