#!/usr/bin/env bash
# Texture-address / L1 counters over a short C3 bench (is a gather kernel
# bound by the per-line address processing rather than by bytes?).  The
# counter list of the box goes to gpurun_out/counters.txt first; one pass
# per block group, each under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
i=0
for set in "TA_TA_BUSY_sum TA_BUSY_avr" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_GATE_EN1_sum" \
           "TD_TD_BUSY_sum TD_BUSY_avr" "SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_ta$i -o run -- \
    python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/pmc_ta$i.json 2> gpurun_out/pmc_ta$i.err
  rc=$?
  echo "pass $i rc=$rc"; tail -2 gpurun_out/pmc_ta$i.err
  case $rc in 0|1) ;; *) exit $rc ;; esac
done
python3 tools/pmc_table.py gpurun_out/pmc_ta1 gpurun_out/pmc_ta2 gpurun_out/pmc_ta3 gpurun_out/pmc_ta4 > gpurun_out/pmc_ta.txt || true
grep -E "k_schur_pairs_c|k_cam_schur_diag|k_lin_point|k_obs_w_rc" gpurun_out/pmc_ta.txt || true
exit 0
