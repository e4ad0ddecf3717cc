#!/usr/bin/env bash
# Round 5: the 64-column register-sweep Cholesky factor (BA_CHOL_SWEEP64=1
# builds: tools/*_sw*, bundleadjustment_amd/ab/libba_sw.so) against the
# four-sub-panel factor — probes, chol_bench (persistent vs per-step bitwise,
# n = 1194 / 6000), the dense GPU tests on the sweep build, the C3 bench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited with $1 — stopping"; exit "$1" ;; esac; }
for b in fullsweep_probe fullsweep_probe_sp; do
  timeout -k 5 60 tools/$b > $OUT/$b.txt 2>&1; rc=$?; cat $OUT/$b.txt; stop_on_fault $rc
done
for b in chol_bench_sw chol_bench_ns; do
  for n in 1194 6000; do
    timeout -k 5 120 tools/$b $n > $OUT/${b}_$n.txt 2>&1; rc=$?
    echo "== $b $n"; grep -E "persistent|factor total|residual|differing" $OUT/${b}_$n.txt; stop_on_fault $rc
  done
done
for b in chol_bench_swst chol_bench; do
  timeout -k 5 120 tools/$b 1194 > $OUT/${b}_1194.txt 2>&1; rc=$?
  echo "== $b 1194"; grep -E "persistent|residual|differing" $OUT/${b}_1194.txt; stop_on_fault $rc
done
BA_HIP_LIB=bundleadjustment_amd/ab/libba_sw.so timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_blocks.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread \
  -k "persistent or solve_matches or c3_first or many_cameras or jfree_blocks or c4_shard or bitwise or compact" \
  > $OUT/pytest_dense_sw.log 2>&1
rc=$?; tail -3 $OUT/pytest_dense_sw.log; stop_on_fault $rc
[ $rc = 0 ] || exit 1
bash tools/ab_bench.sh bundleadjustment_amd/ab/libba_sw.so 2>&1 | tee $OUT/ab_c3.txt
