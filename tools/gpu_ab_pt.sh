set -u
cd "${GRAFT_REPO_ROOT}"
echo "== C3"; timeout -k 10 400 bash tools/ab_bench.sh abtmp/libba_hip_pt8.so abtmp/libba_hip_pt32.so || exit $?
echo "== C5 shard ITERATIVE_SCHUR MIXED_FP32"
BENCH_ARGS="--config c5 --scale 0.125 --linear-solver iterative --precision MIXED_FP32 --steps 10 --warmup 2" \
  timeout -k 10 600 bash tools/ab_bench.sh abtmp/libba_hip_pt8.so abtmp/libba_hip_pt32.so
