# optimize A/B session: the optimize / parity / settings GPU tests on the in-tree build, then
# tools/ab_optimize.py over the given library builds.
# usage: tools/gpu_opt_ab.sh TAG lib1.so lib2.so ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1; shift
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_optimize.py tests/test_gpu_parity.py tests/test_settings.py tests/test_energy_terms.py -m gpu > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 600 python tools/ab_optimize.py "$@" --rounds 3 > gpurun_out/abopt_$TAG.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/abopt_$TAG.log; exit 1; }
cat gpurun_out/abopt_$TAG.log
echo done
