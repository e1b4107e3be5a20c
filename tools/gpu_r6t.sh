# round-6 session q: the frame inverses in one SIMT pass and the pair precalc split over waves
# (k_step_resub).  optimize() bitwise against the previous build (or not), the optimize
# A/B, the optimize / Sophus / KITTI GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6t
mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
L=ldso_amd/lib/libldso_ba.so
timeout -k 10 300 python tools/opt_cmp.py abl/head2/libldso_ba.so $L > $O/optcmp.log 2>&1 || { echo "optcmp failed"; tail -30 $O/optcmp.log; exit 1; }
tail -2 $O/optcmp.log
timeout -k 10 600 python tools/ab_optimize.py abl/head2/libldso_ba.so $L --rounds 4 --reps 10 > $O/abopt.log 2>&1 || { echo "abopt failed"; tail -30 $O/abopt.log; exit 1; }
cat $O/abopt.log
timeout -k 10 500 $PYT tests/test_optimize.py tests/test_sophus_kat.py tests/test_kitti_geometry.py tests/test_settings.py -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo done
