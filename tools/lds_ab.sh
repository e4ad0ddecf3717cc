#!/usr/bin/env bash
# LDS-pad A/B of the split Cholesky: the flow form at
# n = 6000 (and 3000) built with tile row pads of 66 (default), 68 and 70
# doubles (tools/chol_bench_l<LDP>, -DCHOL_BENCH_NO_PERSIST: the persistent
# kernel's LDS is full at 66 — 68 would need 164456 of 163840 bytes), timed and
# with an LDS counter pass each.  Run from the repo root on the GPU box.
set -u
OUT=${1:-gpurun_out/lds_ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
for L in 66 68 70; do
  for N in 3000 6000; do
    timeout -k 5 120 tools/chol_bench_l$L $N > "$OUT/t_l${L}_$N.txt" 2>&1 || exit $?
    timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES --output-format csv \
      -d "$OUT/p_l${L}_$N" -o run -- tools/chol_bench_l$L $N > "$OUT/p_l${L}_$N.log" 2>&1 || exit $?
  done
done
for L in 66 68 70; do
  for N in 3000 6000; do
    echo "== LDP=$L n=$N"
    grep -E "factor flow" "$OUT/t_l${L}_$N.txt" | tail -3
    python3 tools/pmc_table.py "$OUT/p_l${L}_$N" | grep -E "k_chol_flow|k_chol_upd"
  done
done
