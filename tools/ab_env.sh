#!/usr/bin/env bash
# A/B: the default C3 bench under alternative environment settings, interleaved.
#   tools/ab_env.sh "BA_CAM_PT=0" "BA_CAM_PT=1"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for round in 1 2; do
  for e in "$@"; do
    out=$(env $e timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} 2>/dev/null) || { echo "$e failed"; exit 1; }
    echo "$e $(echo "$out" | grep -o '"value": [0-9.]*\|avg_launch_ms": [0-9.]*' | tr '\n' ' ')"
  done
done
