#!/usr/bin/env bash
# C4 at full size on ONE GPU (1k cams x 1M pts x 10M obs): the north-star's
# ">= 10x Ceres-CPU LM-iteration time at 1k cams / 10M obs on one MI355X"
# check, with the CPU restatement timed on the host cores (bounded sample).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u bench.py --config c4 --scale 1.0 --steps 3 --warmup 1 --cpu-seconds 20 \
  > gpurun_out/c4full_dense.json 2> gpurun_out/c4full_dense.err || exit $?
cat gpurun_out/c4full_dense.json
timeout -k 10 600 python3 -u bench.py --config c4 --scale 1.0 --steps 3 --warmup 1 --linear-solver iterative \
  --no-cpu-baseline > gpurun_out/c4full_pcg.json 2> gpurun_out/c4full_pcg.err || exit $?
cat gpurun_out/c4full_pcg.json
