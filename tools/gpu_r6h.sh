# round-6 session h: the host stitch forming G_i itself (k_point_sc's gather + SYRK fused into
# k_stitch_host).  Parity first (the fused-vs-slab bitwise test, the stitch paths, a bitwise
# comparison with the previous build), then the pass / optimize A/B, then the whole GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6h
mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
L=ldso_amd/lib/libldso_ba.so
timeout -k 10 400 $PYT tests/test_gpu_parity.py -m gpu -k "fused_schur or stitch_paths" > $O/first.log 2>&1 || { echo "first tests failed"; tail -60 $O/first.log; exit 1; }
tail -2 $O/first.log
timeout -k 10 300 python tools/cmp_libs.py abl/head/libldso_ba.so $L > $O/cmp.log 2>&1 || { echo "cmp failed"; tail -30 $O/cmp.log; exit 1; }
tail -5 $O/cmp.log
timeout -k 10 600 python tools/ab_libs.py abl/head/libldso_ba.so $L $L:14=0 --rounds 3 > $O/ab64.log 2>&1 || { echo "ab64 failed"; tail -30 $O/ab64.log; exit 1; }
cat $O/ab64.log
timeout -k 10 400 python tools/ab_libs.py abl/head/libldso_ba.so $L --windows 1 --rounds 3 > $O/ab1.log 2>&1 || { echo "ab1 failed"; tail -30 $O/ab1.log; exit 1; }
cat $O/ab1.log
timeout -k 10 500 python tools/ab_optimize.py abl/head/libldso_ba.so $L --rounds 3 --reps 10 > $O/abopt.log 2>&1 || { echo "abopt failed"; tail -30 $O/abopt.log; exit 1; }
cat $O/abopt.log
timeout -k 10 900 $PYT tests -m gpu > $O/gpu_tests.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/gpu_tests.log | head; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
echo done
