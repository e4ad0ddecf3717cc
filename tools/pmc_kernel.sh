#!/usr/bin/env bash
# SQ / LDS counter passes over a short bench run (per-kernel wave-cycle and
# LDS breakdown).  Each pass has its own time limit; a pass that fails for a
# counter-name reason (exit 1) does not stop the others, anything else does.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES" \
           "GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_k$i -o run -- \
    python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/pmc_k$i.json 2> gpurun_out/pmc_k$i.err
  rc=$?
  echo "pass $i rc=$rc"
  case $rc in 0|1) ;; *) exit $rc ;; esac
done
python3 tools/pmc_table.py gpurun_out/pmc_k1 gpurun_out/pmc_k2 gpurun_out/pmc_k3 || true
