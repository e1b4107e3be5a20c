# round-6 session b: the GPU suite (settings / optimize / Sophus-dependent tests first), smoke, the
# bench line, the FETCH_SIZE calibration probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_settings.py tests/test_optimize.py tests/test_kitti_geometry.py -m gpu > gpurun_out/pytest_opt_b.log 2>&1 || { echo "first tests failed"; tail -60 gpurun_out/pytest_opt_b.log; exit 1; }
tail -2 gpurun_out/pytest_opt_b.log
timeout -k 10 900 $PYT tests -m gpu > gpurun_out/pytest_b.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_b.log; exit 1; }
tail -2 gpurun_out/pytest_b.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_b.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_b.log; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err || { echo "bench failed"; tail -20 gpurun_out/bench_b.err; exit 1; }
python -c "import json; d = json.load(open('gpurun_out/bench_b.json')); r = d['roofline']; print('value', d['value'], 'ms', d['ms_per_step'], 'frac', r['frac'], 'frac_step', r['frac_step'], 'wall', r['frac_step_wall'], d['kernel_ms_per_step'], 'opt1', d['single_window']['optimize_all_its']['ms_per_optimize'])"
bash tools/gpu_fetch_probe.sh b
echo done
