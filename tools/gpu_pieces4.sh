# pieces k_linearize: A/B of occupancy / box-stride variants, PMC of the best two
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pc4}
timeout -k 10 500 python tools/ab_libs.py abl/base/libldso_ba.so abl/mb4/libldso_ba.so abl/s120/libldso_ba.so abl/s104mb5/libldso_ba.so --rounds 3 > gpurun_out/ablibs_$TAG.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/ablibs_$TAG.log; exit 1; }
cat gpurun_out/ablibs_$TAG.log
bash tools/gpu_pmc_ab.sh $TAG abl/mb4/libldso_ba.so abl/s120/libldso_ba.so
