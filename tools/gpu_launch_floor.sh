# launch-floor probe (tools/launch_floor.hip): HIP events and rocprofv3 kernel durations
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 60 ./tools/launch_floor > gpurun_out/launch_floor.log 2>&1 || { echo "probe failed"; cat gpurun_out/launch_floor.log; exit 1; }
cat gpurun_out/launch_floor.log
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_lf -o run --output-format csv -- ./tools/launch_floor > gpurun_out/prof_lf.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_lf.log; exit 1; }
cat gpurun_out/prof_lf/run_kernel_stats.csv
