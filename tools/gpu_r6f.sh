# round-6 session f: k_solve_fast scheduling A/B -- wave 0's panel at s_setprio 3, wave 4 (wave 0's
# SIMD partner) out of the trailing update, both -- k_solve_fast alone, then optimize(6).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6f
O=gpurun_out/r6f
timeout -k 10 500 python tools/solve_ab.py abl/base/libldso_ba.so abl/prio/libldso_ba.so abl/skip4/libldso_ba.so abl/both/libldso_ba.so --rounds 3 > $O/solve_ab.log 2>&1 || { echo "solve ab failed"; tail -30 $O/solve_ab.log; exit 1; }
grep BEST $O/solve_ab.log
timeout -k 10 600 python tools/ab_optimize.py abl/base/libldso_ba.so abl/prio/libldso_ba.so abl/skip4/libldso_ba.so abl/both/libldso_ba.so --rounds 3 --reps 10 > $O/abopt.log 2>&1 || { echo "abopt failed"; tail -30 $O/abopt.log; exit 1; }
cat $O/abopt.log
echo done
