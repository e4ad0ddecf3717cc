#!/usr/bin/env bash
# Kernel stats at C3 for the fused diagonal launch and the separate one.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s
export TMPDIR=/tmp
for lib in libba_hip.so ab/libba_nodiag.so; do
  tag=$(basename $lib .so)
  BA_HIP_LIB=bundleadjustment_amd/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s/prof_$tag -o run --output-format csv -- \
    python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/s/prof_$tag.json 2>&1
  rc=$?; echo "$tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
