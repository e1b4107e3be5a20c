# k_stitch_host's Top half on the side stream (default) vs the whole stitch after k_point_sc
# (LDSO_BA_NO_STITCH_OVERLAP=1), same library: the parity / optimize GPU tests, then the bench
# headline and tools/ab_optimize.py interleaved.   usage: tools/gpu_overlap_ab.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_gpu_parity.py tests/test_optimize.py tests/test_settings.py -m gpu > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
for r in 1 2 3; do
  for off in 1 0; do
    LDSO_BA_NO_STITCH_OVERLAP=$off timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu --no-secondary --no-tracker > gpurun_out/ovb_${TAG}.json 2> gpurun_out/ovb_${TAG}.err || { echo "bench failed"; tail -20 gpurun_out/ovb_${TAG}.err; exit 1; }
    python -c "import json; d = json.load(open('gpurun_out/ovb_${TAG}.json')); print('no_overlap=$off', 'ms_per_step %.4f' % d['ms_per_step'], 'klin_us %.1f' % d['roofline']['avg_launch_us'], d['kernel_ms_per_step'])" | tee -a gpurun_out/ovb_${TAG}.log
  done
done
for off in 1 0; do
  LDSO_BA_NO_STITCH_OVERLAP=$off timeout -k 10 400 python tools/ab_optimize.py ldso_amd/lib/libldso_ba.so --rounds 3 > gpurun_out/ovo_${TAG}_$off.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/ovo_${TAG}_$off.log; exit 1; }
  echo "no_overlap=$off"; tail -3 gpurun_out/ovo_${TAG}_$off.log
done
echo done
