set -u
cd "${GRAFT_REPO_ROOT:-.}"
TESTS=1 PROF3=0 PROF=0 AB="BA_PS_DMA=1" bash tools/gpu_iter2.sh || exit $?
AB="- BA_DIAG_IN_PAIRS=1 BA_FOLD_IN_PAIRS=0" ROUNDS=3 KTOP=10 bash tools/gpu_ab_c3.sh || exit $?
AB="- BA_PS_DMA=1" ROUNDS=2 PROF=0 BENCH_ARGS="--workload c4 --scale 0.125" bash tools/gpu_ab_c3.sh
