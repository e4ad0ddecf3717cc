#!/usr/bin/env bash
# PMC passes per workload (C3, C4 shard, C5 shard): FETCH_SIZE and WRITE_SIZE
# in separate passes (HBM bytes per launch, FETCH x2 on gfx950) and one SQ
# pass with the LDS counters.  Each pass runs under its own time limit; a
# pass that fails for a counter-name reason (exit 1) does not stop the rest.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
export TMPDIR=/tmp
SQSET="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU"
# WL: the workloads (default all three), e.g. WL="c3"
WL=${WL:-"c3,c4s --workload c4 --scale 0.125,c5s --workload c5 --scale 0.125"}
IFS=, read -ra WLS <<< "$WL"
for w in "${WLS[@]}"; do
  set -- $w; tag=$1; shift
  for pass in FETCH_SIZE WRITE_SIZE SQ; do
    ctr=$pass; [ $pass = SQ ] && ctr=$SQSET
    timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_${tag}_$pass -o run -- \
      python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > $OUT/pmc_${tag}_$pass.json 2> $OUT/pmc_${tag}_$pass.err
    rc=$?
    echo "$tag $pass rc=$rc"
    case $rc in 0|1) ;; *) exit $rc ;; esac
  done
  python3 tools/pmc_summary.py $OUT/pmc_${tag}_FETCH_SIZE $OUT/pmc_${tag}_WRITE_SIZE $OUT/pmc_${tag}.json > $OUT/pmc_${tag}_hbm.txt || true
  python3 tools/pmc_table.py $OUT/pmc_${tag}_SQ > $OUT/pmc_${tag}_sq.txt || true
  echo "== $tag"; cat $OUT/pmc_${tag}_hbm.txt
done
exit 0
