# A/B of k_stitch_sum batch sizes (tools/build_ab.sh builds), one window and 64 windows
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L="abl/base/libldso_ba.so abl/b48/libldso_ba.so abl/b42/libldso_ba.so"
timeout -k 10 400 python tools/ab_libs.py $L --windows 1 --rounds 3 > gpurun_out/ab_sum1.log 2>&1 || { echo "ab1 failed"; tail -30 gpurun_out/ab_sum1.log; exit 1; }
cat gpurun_out/ab_sum1.log
timeout -k 10 400 python tools/ab_libs.py $L --windows 64 --rounds 3 > gpurun_out/ab_sum64.log 2>&1 || { echo "ab64 failed"; tail -30 gpurun_out/ab_sum64.log; exit 1; }
cat gpurun_out/ab_sum64.log
