# A/B session: parity of each abl/<name> build on the GPU parity suite, then interleaved timings.
# usage: tools/gpu_ab.sh TAG name1 name2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1; shift
for n in "$@"; do
  LDSO_BA_LIB=$PWD/abl/$n/libldso_ba.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu > gpurun_out/ab_${TAG}_parity_$n.log 2>&1 || { echo "parity failed: $n"; tail -30 gpurun_out/ab_${TAG}_parity_$n.log; exit 1; }
  echo "$n: $(tail -1 gpurun_out/ab_${TAG}_parity_$n.log)"
done
libs=""
for n in "$@"; do libs="$libs abl/$n/libldso_ba.so"; done
timeout -k 10 900 python tools/ab_libs.py $libs --rounds 4 > gpurun_out/ab_${TAG}.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/ab_${TAG}.log; exit 1; }
cat gpurun_out/ab_${TAG}.log
