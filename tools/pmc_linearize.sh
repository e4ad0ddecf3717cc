#!/usr/bin/env bash
# PMC passes for the bench (C3): HBM traffic per kernel (FETCH_SIZE and
# WRITE_SIZE in separate passes, MI355X_MICROARCH.md: FETCH_SIZE x2 on gfx950)
# plus the counter list of the box.  Each pass has its own time limit.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc_$ctr -o run -- \
    python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_$ctr.json 2> gpurun_out/pmc_$ctr.err
done
echo done
