#!/usr/bin/env bash
# Back substitution from the CG's accumulated point products (W.pacc): the
# ITERATIVE_SCHUR tests, then A/B (BA_PCG_PACC=0: J per observation)
# interleaved at C4 (fixed radius, trajectory), the C5 and C4 shards, and the
# C4 kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited with $1 — stopping"; exit "$1" ;; esac; }
timeout -k 10 900 python3 -u -m pytest tests/test_pcg.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread \
  -m gpu > $OUT/i_pytest.log 2>&1
rc=$?; tail -3 $OUT/i_pytest.log; stop_on_fault $rc
[ $rc = 0 ] || exit 1
ab() {   # tag, bench args...
  local tag=$1; shift
  for round in 1 2; do
    for v in 1 0; do
      out=$(BA_PCG_PACC=$v timeout -k 10 300 python3 -u bench.py --no-cpu-baseline "$@" 2>$OUT/i_$tag.err) || { echo "$tag pacc=$v failed"; exit 1; }
      echo "$tag pacc=$v $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); t=d.get("trajectory") or {}; print(d["value"], d["ms_per_step"], t.get("linear_solver_iterations"), t.get("final_cost"))')"
    done
  done
}
ab c4fix --workload c4 --mode fixed --steps 20 --warmup 3
ab c4traj --workload c4 --steps 20 --warmup 2
ab c5s --workload c5 --scale 0.125 --mode fixed --steps 20 --warmup 3
ab c4s --workload c4 --scale 0.125 --mode fixed --steps 20 --warmup 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/i_prof -o run --output-format csv -- \
  python3 -u bench.py --workload c4 --mode fixed --steps 10 --warmup 2 --no-cpu-baseline > $OUT/i_prof.json 2>&1
rc=$?; echo "prof rc=$rc"; stop_on_fault $rc
