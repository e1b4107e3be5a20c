# k_step_resub A/B: the optimize / parity GPU tests on the in-tree build, tools/ab_optimize.py
# over the given builds, then a rocprofv3 kernel trace of one-window optimize per build with
# k_step_resub's durations.   usage: tools/gpu_step_ab.sh TAG lib1.so lib2.so ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1; shift
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 $PYT tests/test_optimize.py tests/test_gpu_parity.py tests/test_settings.py -m gpu > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -2 gpurun_out/pytest_$TAG.log
[ -n "$SKIP_AB" ] || timeout -k 10 600 python tools/ab_optimize.py "$@" --rounds 3 > gpurun_out/abopt_$TAG.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/abopt_$TAG.log; exit 1; }
[ -n "$SKIP_AB" ] || cat gpurun_out/abopt_$TAG.log
export TMPDIR=/tmp
for l in "$@"; do
  n=$(basename $(dirname $l))
  LDSO_BA_LIB=$PWD/$l timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/st_$TAG/$n -o run -- python3 tools/optimize_trace.py 5 1 > gpurun_out/st_${TAG}_$n.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/st_${TAG}_$n.log; exit 1; }
  f=$(ls gpurun_out/st_$TAG/$n/*/run_kernel_trace.csv 2>/dev/null | head -1)
  [ -z "$f" ] && f=$(find gpurun_out/st_$TAG/$n -name '*kernel_trace.csv' | head -1)
  python tools/timeline.py $f 42 > gpurun_out/st_${TAG}_$n.timeline
  python - "$f" "$n" <<'PY'
import csv, re, sys, statistics as S
rows = list(csv.DictReader(open(sys.argv[1])))
d = {}
for r in rows:
    m = re.search(r"(k_[a-z_]+)", r["Kernel_Name"])
    if m: d.setdefault(m.group(1), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(sys.argv[2], {k: round(S.median(v), 2) for k, v in d.items() if k in ("k_step_resub", "k_solve_fast", "k_linearize", "k_point_sc", "k_stitch_host", "k_stitch_host_sum")})
PY
done
echo done
