#!/usr/bin/env bash
# The north-star C4 records on one GPU: C4 at full size
# with ITERATIVE_SCHUR and with DENSE_SCHUR (the reference's solver), each
# with the CPU baseline (oracle/ restatement at 4 threads and at every allowed
# thread), then the 1-rank RCCL communicator with the exchange path forced
# (BA_FORCE_COLLECTIVES=1) next to the communicator-free line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited with $1 — stopping"; exit "$1" ;; esac; }
show() { python3 -c "import json; d=json.load(open('$1')); c=d.get('cpu_baseline') or {}; print('$2', d['value'], d['ms_per_step'], d.get('ms_per_step_median'), d['roofline']['frac'], c.get('value'), (c.get('reference_threads') or {}).get('value'))"; }
timeout -k 10 600 python3 -u bench.py --workload c4 --steps 10 --warmup 2 > $OUT/c4_iter.json 2> $OUT/c4_iter.err
rc=$?; show $OUT/c4_iter.json c4_iterative; stop_on_fault $rc
timeout -k 10 900 python3 -u bench.py --workload c4 --linear-solver dense --steps 10 --warmup 2 > $OUT/c4_dense.json 2> $OUT/c4_dense.err
rc=$?; show $OUT/c4_dense.json c4_dense; stop_on_fault $rc
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/c4_nocomm_$r.json 2> $OUT/c4_nocomm_$r.err
  rc=$?; show $OUT/c4_nocomm_$r.json c4_nocomm_$r; stop_on_fault $rc
  BA_FORCE_COLLECTIVES=1 timeout -k 10 300 python3 -u bench.py --workload c4 --comm --steps 10 --warmup 2 --no-cpu-baseline > $OUT/c4_comm_$r.json 2> $OUT/c4_comm_$r.err
  rc=$?; show $OUT/c4_comm_$r.json c4_comm_forced_$r; stop_on_fault $rc
done
exit 0
