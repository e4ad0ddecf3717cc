#!/usr/bin/env bash
# J-free PCG point pass (k_pcg_point_jf): the PCG tests that reach it, then
# A/B (BA_PCG_JF=0: k_obs_w_rc + k_pcg_point_seg) interleaved at C4 full size
# (fixed radius and trajectory), the C5 shard and the C4 shard, and the
# kernel stats of the C4 fixed-radius run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited with $1 — stopping"; exit "$1" ;; esac; }
timeout -k 10 600 python3 -u -m pytest tests/test_pcg.py -x -q --timeout 300 --timeout-method thread \
  -k "jfree or many_cameras or rank2 or exchange" -s > $OUT/g_pytest.log 2>&1
rc=$?; tail -3 $OUT/g_pytest.log; stop_on_fault $rc
[ $rc = 0 ] || exit 1
ab() {   # tag, bench args...
  local tag=$1; shift
  for round in 1 2; do
    for jf in 1 0; do
      out=$(BA_PCG_JF=$jf timeout -k 10 300 python3 -u bench.py --no-cpu-baseline "$@" 2>$OUT/g_$tag.err) || { echo "$tag jf=$jf failed"; exit 1; }
      echo "$tag jf=$jf $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); t=d.get("trajectory") or {}; print(d["value"], d["ms_per_step"], t.get("linear_solver_iterations"))')"
    done
  done
}
ab c4fix --workload c4 --mode fixed --steps 20 --warmup 3
ab c4traj --workload c4 --steps 20 --warmup 2
ab c5s --workload c5 --scale 0.125 --mode fixed --steps 20 --warmup 3
ab c4s --workload c4 --scale 0.125 --mode fixed --steps 20 --warmup 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/g_prof -o run --output-format csv -- \
  python3 -u bench.py --workload c4 --mode fixed --steps 10 --warmup 2 --no-cpu-baseline > $OUT/g_prof.json 2>&1
rc=$?; echo "prof rc=$rc"; stop_on_fault $rc
find $OUT/g_prof -name "*kernel_stats.csv" | head -3
