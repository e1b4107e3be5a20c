# one GPU session: parity tests, bench, kernel-trace profile, PMC traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-x}
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-secondary > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_$TAG.log; exit 1; }
if [ "${2:-}" = "pmc" ]; then
  timeout -k 10 900 python tools/pmc_traffic.py > gpurun_out/pmc_$TAG.log 2>&1 || { echo "pmc failed"; tail -30 gpurun_out/pmc_$TAG.log; exit 1; }
  tail -30 gpurun_out/pmc_$TAG.log
fi
echo done
