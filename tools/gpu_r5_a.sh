set -u
mkdir -p gpurun_out
timeout -k 5 60 tools/fullsweep_probe > gpurun_out/fullsweep.txt 2>&1; rc=$?; cat gpurun_out/fullsweep.txt
case $rc in 0) ;; *) echo "probe rc=$rc"; exit $rc ;; esac
CPU="" bash tools/gpu_r5_traj.sh
