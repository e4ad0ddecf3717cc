#!/usr/bin/env bash
# The ACC point-step prefetch at the C4 shard (1.25M observations), interleaved
# against the previous form.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BENCH_ARGS="--workload c4 --scale 0.125 --mode fixed" timeout -k 10 600 tools/ab_bench.sh bundleadjustment_amd/ab/libba_head.so || exit 1
BENCH_ARGS="--workload c4 --scale 0.125 --mode fixed" timeout -k 10 600 tools/ab_bench.sh bundleadjustment_amd/ab/libba_head.so || exit 1
