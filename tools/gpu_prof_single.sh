set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_single -o run --output-format csv -- python3 tools/solve_breakdown.py > gpurun_out/prof_single.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_single.log; exit 1; }
python tools/trace_summary.py gpurun_out/prof_single/run_kernel_trace.csv > gpurun_out/single_summary.json
python -c "
import json
for d in json.load(open('gpurun_out/single_summary.json')): print(d['kernel'], d['workgroups'], d['calls'], round(d['avg_us'],1), round(d['median_us'],1))
"
