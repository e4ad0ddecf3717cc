#!/usr/bin/env bash
# C5 shard (fixed radius) kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/o
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/o/prof_c5s -o run --output-format csv -- \
  python3 -u bench.py --workload c5 --scale 0.125 --mode fixed --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/o/prof_c5s.json 2>&1
echo "rc=$?"
