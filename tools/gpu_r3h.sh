# full GPU round on the default build, then write-through record stores A/B (kernel and wall per pass)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_round.sh $1 pmc || exit $?
timeout -k 10 300 python tools/ab_libs.py abl/cur/libldso_ba.so abl/wt/libldso_ba.so --rounds 4 > gpurun_out/ablibs_$1.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/ablibs_$1.log; exit 1; }
cat gpurun_out/ablibs_$1.log
