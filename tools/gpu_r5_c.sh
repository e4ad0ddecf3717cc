#!/usr/bin/env bash
# Round 5 records: ITERATIVE / DENSE along a real LM trajectory at C4 full
# size and the C5 shard with the CPU restatement beside them (roofline.traffic
# from the committed C4 / C5-shard PMC), and the frame-to-frame pose-only
# solves (one 500-obs frame, 64- and 4096-frame batches).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited with $1 — stopping"; exit "$1" ;; esac; }
for o in "64 500" "4096 500" "64 1500"; do
  set -- $o
  timeout -k 10 300 python3 -u tools/bench_f2f.py --batch $1 --obs $2 > $OUT/f2f_b$1_o$2.json 2> $OUT/f2f_b$1_o$2.err
  rc=$?; cat $OUT/f2f_b$1_o$2.json; stop_on_fault $rc
done
CPU="" PMC=0 bash tools/gpu_r5_traj.sh
