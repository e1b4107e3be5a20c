# quick GPU check: parity tests + bench (no CPU leg)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-q}
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench_$TAG.json'))
print('value %.3e res/s  ms/step %.4f' % (d['value'], d['ms_per_step']))
print('kernels', {k: round(v*1e3,1) for k,v in d['kernel_ms_per_step'].items()})
print('roofline frac %.3f achieved %.0f GB/s' % (d['roofline']['frac'], d['roofline']['achieved']))
print('single', d['single_window'])
print('gn batched', d.get('gn_iteration_batched'))
"
