#!/usr/bin/env bash
# A/B of env-selected kernel variants on the default bench (interleaved rounds).
# usage: ab_env.sh "ENV1=1" "ENV2=1 ENV3=0" ...   ("" = default)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for round in 1 2; do
  for v in "" "$@"; do
    out=$(env $v timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} 2>/dev/null) || { echo "[$v] failed"; exit 1; }
    echo "[$v] $(echo "$out" | grep -o '"value": [0-9.]*\|avg_launch_ms": [0-9.]*' | tr '\n' ' ')"
  done
done
