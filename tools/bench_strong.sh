#!/usr/bin/env bash
# One-GPU runs of the strong-scaling workloads: C4 (10M obs, ITERATIVE_SCHUR)
# and the C5 per-GPU shard (12.5M obs, ITERATIVE_SCHUR + MIXED_FP32).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c4_n1.json 2> gpurun_out/bench_c4_n1.err
rc=$?; cat gpurun_out/bench_c4_n1.json; tail -2 gpurun_out/bench_c4_n1.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --config c5 --scale 0.125 --linear-solver iterative --precision MIXED_FP32 \
  --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c5shard.json 2> gpurun_out/bench_c5shard.err
rc=$?; cat gpurun_out/bench_c5shard.json; tail -2 gpurun_out/bench_c5shard.err; exit $rc
