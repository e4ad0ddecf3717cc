#!/usr/bin/env bash
# CG update form A/B (one workgroup up to 1024 cameras vs the grid kernels
# past 256, 64- or 256-thread blocks) at C4 and the C5 shard, then the C5
# shard trajectory record with the CPU restatement.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/p
BENCH_ARGS="--workload c4 --mode fixed" timeout -k 10 900 tools/ab_bench.sh bundleadjustment_amd/ab/libba_u64.so bundleadjustment_amd/ab/libba_u256.so || exit 1
BENCH_ARGS="--workload c5 --scale 0.125 --mode fixed" timeout -k 10 600 tools/ab_bench.sh bundleadjustment_amd/ab/libba_u64.so || exit 1
timeout -k 10 600 python3 -u bench.py --workload c5 --scale 0.125 --steps 20 --warmup 2 > gpurun_out/p/bench_c5s.json 2> gpurun_out/p/bench_c5s.err
echo "c5s rc=$?"
