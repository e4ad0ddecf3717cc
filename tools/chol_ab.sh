#!/bin/bash
# A/B of the dense Cholesky (tools/chol_bench.hip, stamped build): the
# committed csrc (git HEAD, or $BASE_REF) against the working tree.
# Build here (CPU):  tools/chol_ab.sh      Run on the GPU box: tools/chol_ab.sh run
set -e
cd "$(dirname "$0")/.."
if [ "$1" != "run" ]; then
  H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DBA_CHOL_STAMPS"
  rm -rf build_ab/base && mkdir -p build_ab/base/bundleadjustment_amd/csrc build_ab/base/include build_ab/base/tools
  git archive "${BASE_REF:-HEAD}" bundleadjustment_amd/csrc include tools/chol_bench.hip | tar -x -C build_ab/base
  $H -I build_ab/base/bundleadjustment_amd/csrc build_ab/base/tools/chol_bench.hip -o tools/chol_bench_base
  $H -I bundleadjustment_amd/csrc tools/chol_bench.hip -o tools/chol_bench
  exit 0
fi
for n in 1194 598; do
  echo "== base n=$n"; timeout -k 5 60 tools/chol_bench_base $n
  echo "== new n=$n"; timeout -k 5 60 tools/chol_bench $n
done
