# in-tree build: GPU parity suite, then A/B against abl/base (one window and 64 windows)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_th.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_th.log; exit 1; }
tail -1 gpurun_out/pytest_th.log
L="abl/base/libldso_ba.so ldso_amd/lib/libldso_ba.so"
timeout -k 10 400 python tools/ab_libs.py $L --windows 1 --rounds 3 > gpurun_out/ab_th1.log 2>&1 || { echo "ab1 failed"; tail -30 gpurun_out/ab_th1.log; exit 1; }
cat gpurun_out/ab_th1.log
timeout -k 10 400 python tools/ab_libs.py $L --windows 64 --rounds 3 > gpurun_out/ab_th64.log 2>&1 || { echo "ab64 failed"; tail -30 gpurun_out/ab_th64.log; exit 1; }
cat gpurun_out/ab_th64.log
