#!/usr/bin/env bash
# Round-5 end records after the fp32 accumulated-products point step, the
# 256-camera CG-update threshold and the diagonal slices in the pair launch.
# PART A: smoke, C3 with its CPU baseline and kernel stats, the Cholesky
# bench.  PART B: C4 ITERATIVE along the trajectory (CPU restatement) and at
# the fixed radius, the C4 shard, the C4 kernel stats.  (GPU suite:
# profiles/r05_v12_diag_in_pairs_ab.txt; C5 shard: r05_v10_bench_c5s_traj.json;
# C4 DENSE unchanged: 1000 cameras keep the separate diagonal launch.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/final2
mkdir -p $OUT
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited with $1 — stopping"; exit "$1" ;; esac; }
run() {   # tag, timeout, bench args...
  local tag=$1 t=$2; shift 2
  echo "== $tag"
  timeout -k 10 $t python3 -u bench.py "$@" > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err
  local rc=$?
  python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read()); t=d.get("trajectory") or {}; print(sys.argv[2], d["value"], d["ms_per_step"], d.get("ms_per_step_median"), (d.get("cpu_baseline") or {}).get("value"), t.get("linear_solver_iterations"))' $OUT/bench_$tag.json $tag || true
  stop_on_fault $rc
}
if [ "${PART:-A}" = A ]; then
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1
rc=$?; tail -1 $OUT/smoke.txt; stop_on_fault $rc
run c3 300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3 -o run --output-format csv -- \
  python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_c3.json 2>&1
rc=$?; echo "prof c3 rc=$rc"; stop_on_fault $rc
timeout -k 5 120 tools/chol_bench_ns 1194 > $OUT/chol_bench_ns_1194.txt 2>&1; rc=$?; grep -E "persistent factor|differing" $OUT/chol_bench_ns_1194.txt | head -3; stop_on_fault $rc
echo "part A done"
exit 0
fi
run c4_iter 600 --workload c4 --steps 20 --warmup 2
run c4_fixed 300 --workload c4 --mode fixed --steps 20 --warmup 3 --no-cpu-baseline
run c4s 300 --workload c4 --scale 0.125 --mode fixed --steps 20 --warmup 3 --no-cpu-baseline
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c4 -o run --output-format csv -- \
  python3 -u bench.py --workload c4 --mode fixed --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_c4.json 2>&1
rc=$?; echo "prof c4 rc=$rc"; stop_on_fault $rc
echo "part B done"
