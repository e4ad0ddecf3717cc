#!/usr/bin/env bash
# Interleaved A/B of env variants on one box: AB="VAR=a VAR=b ..." (the
# first entry may be "-" for the default), R rounds of the C3 bench each,
# then one rocprofv3 kernel-stats run per variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
stop_on_fault() { case "$1" in 0|1) return 0 ;; *) echo "GPU step exited with $1 — stopping"; exit "$1" ;; esac; }
for r in $(seq 1 ${R:-2}); do
  for v in ${AB}; do
    e=${v//,/ }; [ "$v" = "-" ] && e=""
    timeout -k 10 300 env $e python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/ab_$r.json 2>> $OUT/ab.err
    rc=$?; python3 -c "import json; d=json.load(open('$OUT/ab_$r.json')); print('$v', 'round $r', d['value'], d['ms_per_step'])"; stop_on_fault $rc
  done
done
export TMPDIR=/tmp
i=0
for v in ${AB}; do
  i=$((i+1)); e=${v//,/ }; [ "$v" = "-" ] && e=""
  # (rocprofv3 must exec python3 directly: the variant's variables go in through export)
  ( [ -n "$e" ] && export $e; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/abprof$i -o run -- \
    python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/abprof$i.json 2>> $OUT/ab.err )
  rc=$?; stop_on_fault $rc
  echo "== $v"; python3 tools/kstats.py $OUT/abprof$i/run_kernel_stats.csv 11 > $OUT/abprof$i.txt; head -${K:-8} $OUT/abprof$i.txt
done
