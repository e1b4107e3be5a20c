set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "device_solve or fused or optimize" tests/test_optimize.py > gpurun_out/solve_t1.log 2>&1 || { tail -60 gpurun_out/solve_t1.log; exit 1; }
tail -3 gpurun_out/solve_t1.log
timeout -k 10 300 python tools/solve_ab.py ldso_amd/lib/libldso_ba.so ldso_amd/lib/libldso_ba.so@LDSO_BA_SOLVE_LDS=1
