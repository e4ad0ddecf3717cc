#!/usr/bin/env bash
# Round 5: ITERATIVE_SCHUR / DENSE_SCHUR along a real LM trajectory
# (bench.py --mode trajectory) at C4 full size and the C5 shard, with the
# CPU restatement beside them; then the r+J kernel's PMC (FETCH / WRITE / SQ
# passes) at the same sizes for roofline.traffic and the VALU figure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited with $1 — stopping"; exit "$1" ;; esac; }
run() {   # tag, bench args...
  local tag=$1; shift
  timeout -k 10 600 python3 -u bench.py "$@" > $OUT/traj_$tag.json 2> $OUT/traj_$tag.err
  local rc=$?
  python3 - "$OUT/traj_$tag.json" "$tag" <<'EOF' || true
import json, sys
d = json.loads(open(sys.argv[1]).read())
t = d.get("trajectory") or {}
print(sys.argv[2], d["value"], "ms/it", d["ms_per_step"], "median", d.get("ms_per_step_median"),
      "cg", t.get("linear_solver_iterations"), "stop", t.get("ceres_default_function_tolerance_stop"),
      "cpu", (d.get("cpu_baseline") or {}).get("value"))
EOF
  stop_on_fault $rc
}
run c4_iter --workload c4 --steps ${STEPS:-20} --warmup 2 ${CPU---no-cpu-baseline}
run c4_dense --workload c4 --linear-solver dense --steps ${STEPS:-20} --warmup 2 ${CPU---no-cpu-baseline}
run c5s --workload c5 --scale 0.125 --steps ${STEPS:-20} --warmup 2 ${CPU---no-cpu-baseline}
run c4_fixed --workload c4 --mode fixed --steps 20 --warmup 3 --no-cpu-baseline
[ "${PMC:-1}" = 1 ] || exit 0
export TMPDIR=/tmp
for w in "c4 --workload c4 --mode fixed" "c5s --workload c5 --scale 0.125 --mode fixed"; do
  set -- $w; tag=$1; shift
  for pass in FETCH_SIZE WRITE_SIZE SQ; do
    ctr=$pass; [ $pass = SQ ] && ctr="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU"
    timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_${tag}_$pass -o run -- \
      python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > $OUT/pmc_${tag}_$pass.json 2> $OUT/pmc_${tag}_$pass.err
    rc=$?
    echo "$tag $pass rc=$rc"
    stop_on_fault $rc
  done
  nobs=$(python3 -c "import json; print(json.load(open('$OUT/pmc_${tag}_FETCH_SIZE.json'))['config']['global_obs'])")
  python3 tools/pmc_summary.py $OUT/pmc_${tag}_FETCH_SIZE $OUT/pmc_${tag}_WRITE_SIZE $OUT/pmc_${tag}.json \
    --sq $OUT/pmc_${tag}_SQ --n-obs $nobs > $OUT/pmc_${tag}_hbm.txt || true
  python3 tools/pmc_table.py $OUT/pmc_${tag}_SQ > $OUT/pmc_${tag}_sq.txt || true
  echo "== $tag"; cat $OUT/pmc_${tag}_hbm.txt | head -30
done
exit 0
