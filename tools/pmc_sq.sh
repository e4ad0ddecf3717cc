#!/usr/bin/env bash
# One SQ counter pass over a short bench run (per-kernel wave-cycle breakdown).
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d gpurun_out/pmc_sq -o run -- \
  python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_sq.json 2> gpurun_out/pmc_sq.err
echo done
