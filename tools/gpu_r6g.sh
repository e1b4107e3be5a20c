# round-6 session g: k_solve_fast with the panel's diagonal block mirrored lane-uniformly (no
# readlane on the pivot chain): x bit-identical to the base build, then the solve and optimize A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6g
mkdir -p $O
timeout -k 10 300 python tools/solve_x_cmp.py abl/base/libldso_ba.so abl/mirror/libldso_ba.so abl/mirror_prio/libldso_ba.so > $O/xcmp.log 2>&1 || { echo "xcmp failed"; tail -30 $O/xcmp.log; exit 1; }
cat $O/xcmp.log
timeout -k 10 500 python tools/solve_ab.py abl/base/libldso_ba.so abl/mirror/libldso_ba.so abl/mirror_prio/libldso_ba.so --rounds 3 > $O/solve_ab.log 2>&1 || { echo "solve ab failed"; tail -30 $O/solve_ab.log; exit 1; }
grep BEST $O/solve_ab.log
timeout -k 10 600 python tools/ab_optimize.py abl/base/libldso_ba.so abl/mirror/libldso_ba.so abl/mirror_prio/libldso_ba.so --rounds 3 --reps 10 > $O/abopt.log 2>&1 || { echo "abopt failed"; tail -30 $O/abopt.log; exit 1; }
cat $O/abopt.log
echo done
