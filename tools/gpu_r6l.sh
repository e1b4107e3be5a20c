# round-6 session l: the device GN loop forms the evaluation-point pair terms (PRE_RTll_0 /
# PRE_tTll_0) in its first step only.  Bitwise optimize() outputs against the previous build, the
# optimize A/B, the optimize / Sophus GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6l
mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
L=ldso_amd/lib/libldso_ba.so
timeout -k 10 300 python tools/opt_cmp.py abl/head/libldso_ba.so $L > $O/optcmp.log 2>&1 || { echo "optcmp failed"; tail -30 $O/optcmp.log; exit 1; }
tail -2 $O/optcmp.log
timeout -k 10 600 python tools/ab_optimize.py abl/head/libldso_ba.so $L --rounds 4 --reps 10 > $O/abopt.log 2>&1 || { echo "abopt failed"; tail -30 $O/abopt.log; exit 1; }
cat $O/abopt.log
timeout -k 10 500 $PYT tests/test_optimize.py tests/test_sophus_kat.py tests/test_kitti_geometry.py -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo done
