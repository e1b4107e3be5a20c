# round-6 session c: the changed-path GPU tests, the one-wave solve A/B (k_solve_fast alone, then
# optimize(6)), the whole GPU suite, smoke, the bench line, the FETCH_SIZE calibration probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-c}
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 500 $PYT tests/test_settings.py tests/test_optimize.py tests/test_kitti_geometry.py tests/test_gpu_parity.py -k "settings or optimize or kitti or wave or solve or affine" -m gpu > gpurun_out/pytest_first_$T.log 2>&1 || { echo "first tests failed"; tail -60 gpurun_out/pytest_first_$T.log; exit 1; }
tail -2 gpurun_out/pytest_first_$T.log
L=ldso_amd/lib/libldso_ba.so
timeout -k 10 400 python tools/solve_ab.py $L::13=8 $L::13=1 --rounds 2 > gpurun_out/solve_ab_$T.log 2>&1 || { echo "solve ab failed"; tail -30 gpurun_out/solve_ab_$T.log; exit 1; }
grep BEST gpurun_out/solve_ab_$T.log
timeout -k 10 500 python tools/ab_optimize.py $L:13=8 $L:13=1 --rounds 2 --reps 10 > gpurun_out/abopt_$T.log 2>&1 || { echo "abopt failed"; tail -30 gpurun_out/abopt_$T.log; exit 1; }
cat gpurun_out/abopt_$T.log
timeout -k 10 900 $PYT tests -m gpu > gpurun_out/pytest_$T.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_$T.log; exit 1; }
tail -2 gpurun_out/pytest_$T.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_$T.log; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || { echo "bench failed"; tail -20 gpurun_out/bench_$T.err; exit 1; }
python -c "import json; d = json.load(open('gpurun_out/bench_$T.json')); r = d['roofline']; print('value', d['value'], 'ms', d['ms_per_step'], 'frac', r['frac'], 'frac_step', r['frac_step'], 'wall', r['frac_step_wall'], d['kernel_ms_per_step'], 'opt1', d['single_window']['optimize_all_its']['ms_per_optimize'])"
bash tools/gpu_fetch_probe.sh $T
echo done
