# diagnostics: k_schur_pairs time vs its grid cap (BA_PAIRS_GRID)
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for g in 256 1024 8192; do
  BA_PAIRS_GRID=$g timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pg_$g -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || exit 1
  echo "grid $g: $(python3 tools/kstats.py gpurun_out/pg_$g/run_kernel_stats.csv | grep schur_pairs)"
done
