# round-6 session i: k_linearize without makeImages' gradient compare on frames where the load proved
# it never fires.  Parity (the clamp test, bitwise vs the previous build), the pass A/B, the GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6i
mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
L=ldso_amd/lib/libldso_ba.so
timeout -k 10 400 $PYT tests/test_gpu_parity.py -m gpu -k "gradient_clamp or layout or golden or full_s7" > $O/first.log 2>&1 || { echo "first tests failed"; tail -60 $O/first.log; exit 1; }
tail -2 $O/first.log
timeout -k 10 300 python tools/cmp_libs.py abl/head/libldso_ba.so $L > $O/cmp.log 2>&1 || { echo "cmp failed"; tail -30 $O/cmp.log; exit 1; }
tail -3 $O/cmp.log
timeout -k 10 700 python tools/ab_libs.py abl/head/libldso_ba.so $L --rounds 4 > $O/ab64.log 2>&1 || { echo "ab64 failed"; tail -30 $O/ab64.log; exit 1; }
cat $O/ab64.log
timeout -k 10 900 $PYT tests -m gpu > $O/gpu_tests.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/gpu_tests.log | head; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
echo done
