# round-6 session o: k_solve_fast's panel with only the pivot chain in wave 0 (L / d stores and the
# forward substitution moved to the other waves).  x and optimize() bitwise against the previous
# build, the solve and optimize A/B, the solve / optimize GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6o
mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
L=ldso_amd/lib/libldso_ba.so
timeout -k 10 300 python tools/solve_x_cmp.py abl/head/libldso_ba.so $L > $O/xcmp.log 2>&1 || { echo "xcmp failed"; tail -30 $O/xcmp.log; exit 1; }
tail -2 $O/xcmp.log
timeout -k 10 300 python tools/opt_cmp.py abl/head/libldso_ba.so $L > $O/optcmp.log 2>&1 || { echo "optcmp failed"; tail -30 $O/optcmp.log; exit 1; }
tail -2 $O/optcmp.log
timeout -k 10 500 python tools/solve_ab.py abl/head/libldso_ba.so $L --rounds 3 > $O/solve_ab.log 2>&1 || { echo "solve ab failed"; tail -30 $O/solve_ab.log; exit 1; }
grep BEST $O/solve_ab.log
timeout -k 10 600 python tools/ab_optimize.py abl/head/libldso_ba.so $L --rounds 4 --reps 10 > $O/abopt.log 2>&1 || { echo "abopt failed"; tail -30 $O/abopt.log; exit 1; }
cat $O/abopt.log
timeout -k 10 500 $PYT tests/test_optimize.py tests/test_gpu_parity.py -m gpu -k "solve or optimize or rccl" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo done
