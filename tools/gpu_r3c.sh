# k_linearize no-math ablation A/B; bench timed-region launch time vs step count (clock ramp check)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r3c}
timeout -k 10 300 python tools/ab_libs.py abl/base/libldso_ba.so abl/mb4/libldso_ba.so abl/nomath/libldso_ba.so --rounds 3 > gpurun_out/ablibs_$TAG.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/ablibs_$TAG.log; exit 1; }
cat gpurun_out/ablibs_$TAG.log
for sw in "20 5" "400 100"; do
  set -- $sw
  timeout -k 10 200 python bench.py --steps $1 --warmup $2 --no-cpu --no-tracker --no-secondary > gpurun_out/bench_${TAG}_$1.json 2> gpurun_out/bench_${TAG}_$1.err || { echo "bench failed"; tail -20 gpurun_out/bench_${TAG}_$1.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bench_${TAG}_$1.json'))
print('steps $1 warmup $2: ms/step %.4f  k_linearize timed %.1f us  breakdown %.1f us' % (d['ms_per_step'], d['roofline']['avg_launch_us'], 1e3*d['kernel_ms_per_step']['k_linearize']))"
done
