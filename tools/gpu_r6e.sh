# round-6 session e: k_linearize's Top block with every operand read unconditionally and pipelined
# (abl/toppipe: -DLDSO_TOP_PIPE) -- bitwise comparison with the in-tree build, its parity suite,
# interleaved timing -- plus any further variants named on the command line (abl/<name>).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-e}; shift
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
L=ldso_amd/lib/libldso_ba.so
for v in toppipe "$@"; do
  timeout -k 10 300 python tools/cmp_libs.py $L abl/$v/libldso_ba.so > gpurun_out/cmp_${v}_$T.log 2>&1; echo "$v cmp rc=$?: $(tail -1 gpurun_out/cmp_${v}_$T.log)"
  LDSO_BA_LIB=$PWD/abl/$v/libldso_ba.so timeout -k 10 400 $PYT tests/test_gpu_parity.py tests/test_golden.py tests/test_kitti_geometry.py tests/test_optimize.py -m gpu > gpurun_out/pytest_${v}_$T.log 2>&1 || { echo "$v parity failed"; tail -30 gpurun_out/pytest_${v}_$T.log; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/pytest_${v}_$T.log)"
done
libs="$L"; for v in toppipe "$@"; do libs="$libs abl/$v/libldso_ba.so"; done
timeout -k 10 700 python tools/ab_libs.py $libs --rounds 3 > gpurun_out/ab_$T.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/ab_$T.log; exit 1; }
cat gpurun_out/ab_$T.log
echo done
