set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider 2>&1 | tee gpurun_out/pytest_gpu.log
rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/ab_bench.sh abtmp/libba_hip_pl8.so abtmp/libba_hip_pl32.so
