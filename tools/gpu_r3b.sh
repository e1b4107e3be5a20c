# round 3 (session 2): full GPU suite, bench, rocprof stats, PMC traffic, then the T-stride A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_round.sh $1 pmc || exit $?
timeout -k 10 300 python tools/ab_libs.py abl/mb4/libldso_ba.so abl/t76/libldso_ba.so --rounds 3 > gpurun_out/ablibs_$1.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/ablibs_$1.log; exit 1; }
cat gpurun_out/ablibs_$1.log
