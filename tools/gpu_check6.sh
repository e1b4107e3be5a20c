# Round-6 check session: the GPU suite, smoke and the default bench line on the in-tree build.
# usage: tools/gpu_check6.sh TAG      -> gpurun_out/check_TAG/...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/check_$1
mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 600 $PYT tests -m gpu > $O/gpu_tests.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" $O/gpu_tests.log | head -20; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python -c "import json; d = json.load(open('$O/bench.json')); print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'frac', d['roofline']['frac'], 'klin_us', d['roofline']['avg_launch_us'], 'opt1', d['single_window']['optimize_all_its']['ms_per_optimize'])"
echo done
