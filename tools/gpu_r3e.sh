# headline timing with the S11 leg before vs after it (driver flags)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r3e}
for v in first last first last; do
  extra=""; [ $v = last ] && extra="--s11-last"
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-tracker $extra > gpurun_out/bench_${TAG}_$v.json 2> gpurun_out/bench_${TAG}_$v.err || { echo "bench failed"; tail -20 gpurun_out/bench_${TAG}_$v.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bench_${TAG}_$v.json'))
print('s11 $v: ms/step %.4f  k_linearize timed %.1f us  breakdown %.1f us  s11 %.1f us' % (d['ms_per_step'], d['roofline']['avg_launch_us'], 1e3*d['kernel_ms_per_step']['k_linearize'], d['s11']['k_linearize_us']))"
done
