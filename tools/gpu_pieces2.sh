# pieces k_linearize round 2: parity of the skip variant as the product build, A/B and PMC passes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pc2}
LDSO_BA_LIB=$(realpath abl/pieces8/libldso_ba.so) timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "single_pass or wide_pattern or s11_window" > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 400 python tools/ab_libs.py abl/base/libldso_ba.so abl/pieces/libldso_ba.so abl/pieces8/libldso_ba.so --rounds 3 > gpurun_out/ablibs_$TAG.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/ablibs_$TAG.log; exit 1; }
cat gpurun_out/ablibs_$TAG.log
bash tools/gpu_pmc_ab.sh $TAG abl/base/libldso_ba.so abl/pieces8/libldso_ba.so
