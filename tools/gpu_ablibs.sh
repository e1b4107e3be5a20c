# A/B library builds on the GPU: tools/gpu_ablibs.sh TAG lib1.so lib2.so ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 600 python tools/ab_libs.py "$@" > gpurun_out/ablibs_$TAG.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/ablibs_$TAG.log; exit 1; }
cat gpurun_out/ablibs_$TAG.log
