#!/usr/bin/env bash
# A/B of the working tree's library against the previous commit's
# (bundleadjustment_amd/ab/libba_head.so), interleaved, at C4 (fixed radius,
# trajectory), the C5 and C4 shards and C3; the PCG tests first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
export TMPDIR=/tmp
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited with $1 — stopping"; exit "$1" ;; esac; }
timeout -k 10 900 python3 -u -m pytest tests/test_pcg.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread \
  -m gpu > $OUT/k_pytest.log 2>&1
rc=$?; tail -2 $OUT/k_pytest.log; stop_on_fault $rc
[ $rc = 0 ] || exit 1
ab() {   # tag, bench args...
  local tag=$1; shift
  for round in 1 2; do
    for lib in bundleadjustment_amd/libba_hip.so bundleadjustment_amd/ab/libba_head.so; do
      out=$(BA_HIP_LIB=$lib timeout -k 10 300 python3 -u bench.py --no-cpu-baseline "$@" 2>$OUT/k_$tag.err) || { echo "$tag $lib failed"; exit 1; }
      echo "$tag $(basename $lib) $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); t=d.get("trajectory") or {}; print(d["value"], d["ms_per_step"], t.get("final_cost"))')"
    done
  done
}
ab c4fix --workload c4 --mode fixed --steps 20 --warmup 3
ab c4traj --workload c4 --steps 20 --warmup 2
ab c5s --workload c5 --scale 0.125 --mode fixed --steps 20 --warmup 3
ab c4s --workload c4 --scale 0.125 --mode fixed --steps 20 --warmup 3
if [ -n "${PROF:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/k_prof -o run --output-format csv -- \
    python3 -u bench.py --workload c4 --mode fixed --steps 10 --warmup 2 --no-cpu-baseline > $OUT/k_prof.json 2>&1
  rc=$?; echo "prof rc=$rc"; stop_on_fault $rc
fi
