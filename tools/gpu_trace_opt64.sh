set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/opt_trace64 -o run -- python3 tools/optimize_trace.py 3 64 > gpurun_out/opt_trace64.log 2>&1 || { tail -20 gpurun_out/opt_trace64.log; exit 1; }
f=$(find gpurun_out/opt_trace64 -name '*kernel_trace.csv' | head -1)
python3 tools/timeline.py $f 30
