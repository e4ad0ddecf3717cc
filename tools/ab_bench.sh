#!/usr/bin/env bash
# A/B: the default C3 bench with alternative library builds (BA_HIP_LIB), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for round in 1 2; do
  for lib in bundleadjustment_amd/libba_hip.so "$@"; do
    out=$(BA_HIP_LIB=$lib timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} 2>/dev/null) || { echo "$lib failed"; exit 1; }
    echo "$lib $(echo "$out" | grep -o '"value": [0-9.]*\|avg_launch_ms": [0-9.]*' | tr '\n' ' ')"
  done
done
