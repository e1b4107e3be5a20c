# final round on the default build, then the light-sync phase A variant (parity + A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_round.sh $1 pmc || exit $?
LDSO_BA_LIB=$(realpath abl/light/libldso_ba.so) timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_marginalization.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$1_light.log 2>&1 || { echo "light pytest failed"; tail -40 gpurun_out/pytest_$1_light.log; exit 1; }
tail -1 gpurun_out/pytest_$1_light.log
timeout -k 10 300 python tools/ab_libs.py abl/cur/libldso_ba.so abl/light/libldso_ba.so --rounds 4 > gpurun_out/ablibs_$1.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/ablibs_$1.log; exit 1; }
cat gpurun_out/ablibs_$1.log
