set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 200 python tools/sys_compare.py abl/old/libldso_ba.so ldso_amd/lib/libldso_ba.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu > gpurun_out/stitch_t.log 2>&1 || { tail -40 gpurun_out/stitch_t.log; exit 1; }
tail -2 gpurun_out/stitch_t.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/opt_trace2 -o run -- python3 tools/optimize_trace.py 5 > gpurun_out/opt_trace2.log 2>&1 || { tail -20 gpurun_out/opt_trace2.log; exit 1; }
f=$(find gpurun_out/opt_trace2 -name '*kernel_trace.csv' | head -1)
python3 tools/timeline.py $f 24
