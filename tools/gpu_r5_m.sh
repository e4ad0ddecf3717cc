#!/usr/bin/env bash
# DENSE_SCHUR point step from the compact W records: GPU tests, then A/B against
# the previous commit's library at C3 (default bench) and C4 DENSE (fixed radius)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_blocks.py tests/test_gpu_configs.py -x -q \
  --timeout 300 --timeout-method thread -m gpu > gpurun_out/m_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/m_pytest.log
[ $rc = 0 ] || exit $rc
bash tools/ab_bench.sh bundleadjustment_amd/ab/libba_head.so
BENCH_ARGS="--workload c4 --linear-solver dense --mode fixed" bash tools/ab_bench.sh bundleadjustment_amd/ab/libba_head.so
