# one-round Top operand staging: parity on the default build, A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r3i}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_marginalization.py tests/test_optimize.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 400 python tools/ab_libs.py abl/cur/libldso_ba.so abl/top2/libldso_ba.so abl/topfull/libldso_ba.so --rounds 4 > gpurun_out/ablibs_$TAG.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/ablibs_$TAG.log; exit 1; }
cat gpurun_out/ablibs_$TAG.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-tracker > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench_$TAG.json'))
print('ms/step %.4f value %.3e k_linearize timed %.1f us frac %.3f breakdown %s' % (d['ms_per_step'], d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], {k: round(1e3*v,1) for k,v in d['kernel_ms_per_step'].items()}))"
