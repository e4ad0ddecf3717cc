#!/usr/bin/env bash
# The ACC point step with its per-point inputs loaded one point ahead (148
# VGPRs, 3 waves per SIMD) against the previous form (96 VGPRs, 5 waves), C4
# and the C5 shard at the fixed radius, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BENCH_ARGS="--workload c4 --mode fixed" timeout -k 10 900 tools/ab_bench.sh bundleadjustment_amd/ab/libba_head.so || exit 1
BENCH_ARGS="--workload c5 --scale 0.125 --mode fixed" timeout -k 10 600 tools/ab_bench.sh bundleadjustment_amd/ab/libba_head.so || exit 1
