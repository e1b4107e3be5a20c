# bench.py's headline (timed region as the driver runs it) for several library builds, interleaved:
#   bash tools/ab_bench.sh TAG ROUNDS lib1.so lib2.so ...   -> gpurun_out/abbench_TAG.log
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1; R=$2; shift 2
for r in $(seq 1 $R); do
  for l in "$@"; do
    LDSO_BA_LIB=$PWD/$l timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu --no-secondary --no-tracker > gpurun_out/abbench_${TAG}.json 2> gpurun_out/abbench_${TAG}.err || { echo "bench failed: $l"; tail -20 gpurun_out/abbench_${TAG}.err; exit 1; }
    python -c "import json; d = json.load(open('gpurun_out/abbench_${TAG}.json')); print('$l', 'ms_per_step %.4f' % d['ms_per_step'], 'value %.3e' % d['value'], 'klin_us %.1f' % d['roofline']['avg_launch_us'], 'frac %.3f' % d['roofline']['frac'])" | tee -a gpurun_out/abbench_${TAG}.log
  done
done
