#!/usr/bin/env bash
# ITERATIVE_SCHUR benches (1 GPU): C3, the C4 and C5 per-GPU shards; DENSE_SCHUR C4 shard for comparison.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 ${TLIM:-400} python3 -u bench.py --no-cpu-baseline "$@" > $OUT/$name.json 2> $OUT/$name.err
  local rc=$?; cat $OUT/$name.json; tail -2 $OUT/$name.err; return $rc
}
run pcg_c3 --steps 10 --warmup 2 --linear-solver iterative &&
run pcg_c3_jac --steps 10 --warmup 2 --linear-solver iterative --preconditioner JACOBI &&
run pcg_c4 --config c4 --scale 0.125 --steps 5 --warmup 1 --linear-solver iterative &&
run dense_c4 --config c4 --scale 0.125 --steps 5 --warmup 1 &&
run pcg_c5 --config c5 --scale 0.125 --steps 3 --warmup 1 --linear-solver iterative &&
run pcg_c5_mixed --config c5 --scale 0.125 --steps 3 --warmup 1 --linear-solver iterative --precision MIXED_FP32
