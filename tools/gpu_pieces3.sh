# pieces k_linearize: parity (product build), A/B of the variants
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pc3}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 500 python tools/ab_libs.py abl/base/libldso_ba.so abl/pieces/libldso_ba.so abl/pieces8/libldso_ba.so abl/mb4/libldso_ba.so --rounds 3 > gpurun_out/ablibs_$TAG.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/ablibs_$TAG.log; exit 1; }
cat gpurun_out/ablibs_$TAG.log
