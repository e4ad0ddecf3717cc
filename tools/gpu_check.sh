#!/usr/bin/env bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace.
# Every GPU step has its own time limit; a fault / abort / timeout stops the
# script (no further GPU work), a plain test failure does not.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
STEPS=${STEPS:-20}
stop_on_fault() {  # $1 = exit status of a GPU step
  case "$1" in
    0|1) return 0 ;;
    *) echo "GPU step exited with $1 — stopping"; exit "$1" ;;
  esac
}
echo "== rocm-smi"; (rocm-smi --showproductname 2>&1 | head -20) || true
if [ "${CHOL:-0}" = "1" ]; then
  echo "== chol_bench (stamped build: factor + dataflow back substitution, residual check)"
  for n in 1194 3000; do
    timeout -k 10 120 tools/chol_bench $n > $OUT/chol_bench_$n.txt 2>&1
    rc=$?; tail -4 $OUT/chol_bench_$n.txt; stop_on_fault $rc
  done
fi
echo "== pytest -m gpu"
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -30 $OUT/pytest_gpu.log; stop_on_fault $rc
echo "== smoke"
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -5 $OUT/smoke.log; stop_on_fault $rc
echo "== bench"
timeout -k 10 600 python3 -u bench.py --steps "$STEPS" --warmup 3 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; tail -5 $OUT/bench.err; stop_on_fault $rc
echo "== bench through torch.distributed.run with an RCCL communicator (1 rank)"
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 1 --comm --no-cpu-baseline > $OUT/bench_comm.json 2> $OUT/bench_comm.err
rc=$?; cat $OUT/bench_comm.json; tail -3 $OUT/bench_comm.err; stop_on_fault $rc
echo "== rocprofv3 kernel trace"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err
rc=$?; tail -3 $OUT/prof.err; stop_on_fault $rc
find $OUT/prof -name "*stats*" | head
if [ "${PMC:-0}" = "1" ]; then
  echo "== rocprofv3 PMC (separate passes: FETCH_SIZE, WRITE_SIZE)"
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_$ctr -o run -- \
      python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/pmc_$ctr.json 2> $OUT/pmc_$ctr.err
    rc=$?; tail -2 $OUT/pmc_$ctr.err; stop_on_fault $rc
  done
fi
exit 0
