#!/usr/bin/env bash
# the forced one-rank RCCL exchange (--comm,
# BA_FORCE_COLLECTIVES=1) against the communicator-free solve along the C4
# trajectory, interleaved twice; then the C5-shard trajectory with the CPU
# restatement (ITERATIVE_SCHUR at C5 scale) beside it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited with $1 — stopping"; exit "$1" ;; esac; }
summ() { python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read()); t=d.get("trajectory") or {}; print(sys.argv[2], d["value"], d["ms_per_step"], d.get("ms_per_step_median"), t.get("linear_solver_iterations"), t.get("final_cost"), (d.get("cpu_baseline") or {}).get("value"))' "$@"; }
for r in 1 2; do
  BA_FORCE_COLLECTIVES=1 timeout -k 10 300 python3 -u bench.py --workload c4 --comm --steps 20 --warmup 2 --no-cpu-baseline \
    > $OUT/j_c4traj_comm_$r.json 2> $OUT/j_c4traj_comm_$r.err
  rc=$?; stop_on_fault $rc; summ $OUT/j_c4traj_comm_$r.json comm_$r
  timeout -k 10 300 python3 -u bench.py --workload c4 --steps 20 --warmup 2 --no-cpu-baseline \
    > $OUT/j_c4traj_nocomm_$r.json 2> $OUT/j_c4traj_nocomm_$r.err
  rc=$?; stop_on_fault $rc; summ $OUT/j_c4traj_nocomm_$r.json nocomm_$r
done
timeout -k 10 600 python3 -u bench.py --workload c5 --scale 0.125 --steps 20 --warmup 2 \
  > $OUT/j_c5s_traj_cpu.json 2> $OUT/j_c5s_traj_cpu.err
rc=$?; stop_on_fault $rc; summ $OUT/j_c5s_traj_cpu.json c5s_cpu
