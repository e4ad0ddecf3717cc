#!/usr/bin/env bash
# end_step attribution: stamped chol_bench (V stores split) and a build
# without the V stores (diagnostic timing only: the workers read stale V)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited with $1 — stopping"; exit "$1" ;; esac; }
for b in chol_bench chol_bench_ns chol_bench_nov; do
  timeout -k 5 120 tools/$b 1194 > $OUT/f_${b}_1194.txt 2>&1; rc=$?
  echo "== $b"; grep -E "persistent|V clean|differing" $OUT/f_${b}_1194.txt | head -12; stop_on_fault $rc
done
