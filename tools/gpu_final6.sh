# Round-6 measurement session on the in-tree build: the GPU suite, smoke, the default bench line,
# a rocprofv3 kernel trace of the bench (--kernel-trace --stats) and the HBM traffic of
# k_linearize from separate --pmc passes (tools/pmc_traffic.py, provenance: session + lib sha256).
# usage: tools/gpu_final6.sh TAG      -> gpurun_out/final_TAG/...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/final_$1
mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 600 $PYT tests -m gpu > $O/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python -c "import json; d = json.load(open('$O/bench.json')); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'frac', d['roofline']['frac'], 'klin_us', d['roofline']['avg_launch_us'])"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-secondary > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
python tools/prof_summary.py $O/prof $O/prof_bench_kernels.json "round 6 $1: bench.py --steps 20 --warmup 3 --no-cpu --no-secondary" > /dev/null
python -c "
import json; d = json.load(open('$O/prof_bench_kernels.json'))
ks = d.get('kernels', d)
for k, v in sorted(ks.items(), key=lambda kv: -kv[1].get('total_us', 0) if isinstance(kv[1], dict) else 0)[:8]: print(k, v)
"
LDSO_PMC_SESSION="round 6 $1" timeout -k 10 900 python tools/pmc_traffic.py > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -30 $O/pmc.log; exit 1; }
cp gpurun_out/pmc_k_linearize.json $O/pmc_k_linearize.json
python -c "import json; d = json.load(open('$O/pmc_k_linearize.json')); print({k: d[k] for k in ('FETCH_SIZE_KiB_per_launch', 'WRITE_SIZE_KiB_per_launch', 'hbm_bytes_per_launch', 'hbm_bytes_per_gather_residual', 'lib_sha256')})"
echo done
