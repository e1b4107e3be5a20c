# bench with the gather count moved after the timed region: the driver's flags and a long run
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r3d}
for sw in "20 5" "400 100" "20 5"; do
  set -- $sw
  timeout -k 10 200 python bench.py --steps $1 --warmup $2 --no-cpu --no-tracker > gpurun_out/bench_${TAG}_$1.json 2> gpurun_out/bench_${TAG}_$1.err || { echo "bench failed"; tail -20 gpurun_out/bench_${TAG}_$1.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bench_${TAG}_$1.json'))
print('steps $1 warmup $2: ms/step %.4f  k_linearize timed %.1f us  breakdown %.1f us  s11 %.1f us' % (d['ms_per_step'], d['roofline']['avg_launch_us'], 1e3*d['kernel_ms_per_step']['k_linearize'], d['s11']['k_linearize_us']))"
done
