# round-6 GPU session: the tests named in $FIRST (default: the KITTI-geometry tests) first, then the whole GPU suite, smoke, a bench line.
# usage: FIRST="tests/x.py ..." tools/gpu_r6.sh TAG [bench|prof|pmc]...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-x}; shift
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 400 $PYT ${FIRST:-tests/test_kitti_geometry.py} -m gpu > gpurun_out/pytest_opt_$TAG.log 2>&1 || { echo "optimize tests failed"; tail -60 gpurun_out/pytest_opt_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_opt_$TAG.log
timeout -k 10 900 $PYT tests -m gpu > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
for step in "$@"; do
  case $step in
    bench)
      timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
      cat gpurun_out/bench_$TAG.json ;;
    prof)
      export TMPDIR=/tmp
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-secondary > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_$TAG.log; exit 1; } ;;
    mgpu)  # the N > 1 launch rehearsed on one GPU: bench.py starts its 2 ranks itself
      LDSO_BENCH_SHARE_GPU=1 timeout -k 10 600 python bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu --no-tracker --no-secondary > gpurun_out/bench2_$TAG.json 2> gpurun_out/bench2_$TAG.err || { echo "bench --gpus 2 failed"; tail -20 gpurun_out/bench2_$TAG.err; exit 1; }
      python -c "import json; d = json.load(open('gpurun_out/bench2_$TAG.json')); print('n_gpus', d['n_gpus'], 'value', d['value'], 'sharded_window', json.dumps(d.get('sharded_window'))[:300])" ;;
    pmc)
      timeout -k 10 900 python tools/pmc_traffic.py > gpurun_out/pmc_$TAG.log 2>&1 || { echo "pmc failed"; tail -30 gpurun_out/pmc_$TAG.log; exit 1; }
      tail -30 gpurun_out/pmc_$TAG.log ;;
  esac
done
echo done
