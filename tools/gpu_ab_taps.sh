set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in t1 t2; do
  LDSO_BA_LIB=abl/$v/libldso_ba.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "single_pass or multi_window or image_layout or chunk" > gpurun_out/par_$v.log 2>&1 || { echo "parity $v failed"; tail -30 gpurun_out/par_$v.log; exit 1; }
  tail -1 gpurun_out/par_$v.log
done
timeout -k 10 600 python tools/ab_libs.py abl/base/libldso_ba.so abl/t1/libldso_ba.so abl/t2/libldso_ba.so abl/t2w5/libldso_ba.so --rounds 3 > gpurun_out/ab_taps.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/ab_taps.log; exit 1; }
cat gpurun_out/ab_taps.log
