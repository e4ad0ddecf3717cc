#!/usr/bin/env bash
# Cholesky tail changes: chol_bench (stamped + plain; n = 1194, 1152 with a
# full last block, 6000 split), the dense GPU tests, and the C3 bench A/B
# against the previous commit's library (bundleadjustment_amd/ab/libba_head.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited with $1 — stopping"; exit "$1" ;; esac; }
for b in chol_bench_ns chol_bench; do
  for n in 1194 1152 6000; do
    [ $b = chol_bench ] && [ $n = 6000 ] && continue
    timeout -k 5 120 tools/$b $n > $OUT/${b}_$n.txt 2>&1; rc=$?
    echo "== $b $n"; grep -E "persistent|factor total|residual|differing|critical cycles|tail" $OUT/${b}_$n.txt | head -12; stop_on_fault $rc
  done
done
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_blocks.py tests/test_gpu_configs.py -x -q \
  --timeout 300 --timeout-method thread \
  -k "persistent or solve_matches or c3_first or many_cameras or jfree_blocks or c4_shard or bitwise or compact" \
  > $OUT/pytest_dense.log 2>&1
rc=$?; tail -3 $OUT/pytest_dense.log; stop_on_fault $rc
[ $rc = 0 ] || exit 1
bash tools/ab_bench.sh bundleadjustment_amd/ab/libba_head.so 2>&1 | tee $OUT/ab_c3.txt
