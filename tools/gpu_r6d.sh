# round-6 session d: k_solve_fast per-phase stamps (diagnostic builds) and the strip trailing update
# (abl/stripsx: -DLDSO_SOLVE_STRIPS) -- its parity (the solve and optimize tests on that library),
# the solve A/B and the one-window optimize A/B against the in-tree build.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-d}
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 python tools/solve_stamps.py abl/stamps/libldso_ba.so abl/strips/libldso_ba.so > gpurun_out/solve_stamps_$T.log 2>&1 || { echo "stamps failed"; tail -30 gpurun_out/solve_stamps_$T.log; exit 1; }
head -80 gpurun_out/solve_stamps_$T.log
LDSO_BA_LIB=$PWD/abl/stripsx/libldso_ba.so timeout -k 10 400 $PYT tests/test_gpu_parity.py tests/test_optimize.py -k "solve or optimize or iterate" -m gpu > gpurun_out/pytest_strips_$T.log 2>&1 || { echo "strips parity failed"; tail -40 gpurun_out/pytest_strips_$T.log; exit 1; }
tail -2 gpurun_out/pytest_strips_$T.log
L=ldso_amd/lib/libldso_ba.so
timeout -k 10 400 python tools/solve_ab.py $L abl/stripsx/libldso_ba.so --rounds 3 > gpurun_out/solve_ab_$T.log 2>&1 || { echo "solve ab failed"; tail -30 gpurun_out/solve_ab_$T.log; exit 1; }
grep BEST gpurun_out/solve_ab_$T.log
timeout -k 10 500 python tools/ab_optimize.py $L abl/stripsx/libldso_ba.so --rounds 3 --reps 10 > gpurun_out/abopt_$T.log 2>&1 || { echo "abopt failed"; tail -30 gpurun_out/abopt_$T.log; exit 1; }
cat gpurun_out/abopt_$T.log
echo done
