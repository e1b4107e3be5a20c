# two-steps-ahead footprint pieces: parity + A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r3k}
LDSO_BA_LIB=$(realpath abl/d2/libldso_ba.so) timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_marginalization.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python tools/ab_libs.py abl/cur/libldso_ba.so abl/d2/libldso_ba.so --rounds 4 > gpurun_out/ablibs_$TAG.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/ablibs_$TAG.log; exit 1; }
cat gpurun_out/ablibs_$TAG.log
