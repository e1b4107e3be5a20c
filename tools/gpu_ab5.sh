# Round-5 A/B session: the GPU suite on the in-tree build, then interleaved timings and the HBM
# traffic counters (FETCH_SIZE, WRITE_SIZE: separate rocprofv3 passes) of k_linearize / k_point_sc
# for each variant.  A variant is abl/<name>[:tuning], e.g. "base" "rec48" "base:10=1".
# usage: tools/gpu_ab5.sh TAG variant1 variant2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1; shift
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $PYT tests -m gpu > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
# each variant's parity on the GPU parity suite (the library given by LDSO_BA_LIB)
for v in "$@"; do
  n=${v%%:*}; t=${v#$n}; t=${t#:}
  [ -f abl/$n/libldso_ba.so ] || continue
  LDSO_AB_TUNE=$t LDSO_BA_LIB=$PWD/abl/$n/libldso_ba.so timeout -k 10 300 $PYT tests/test_gpu_parity.py tests/test_optimize.py -m gpu > gpurun_out/pytest_${TAG}_$n.log 2>&1 || { echo "parity failed: $v"; tail -30 gpurun_out/pytest_${TAG}_$n.log; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/pytest_${TAG}_$n.log)"
done
libs=""
for v in "$@"; do n=${v%%:*}; t=${v#$n}; libs="$libs abl/$n/libldso_ba.so$t"; done
timeout -k 10 900 python tools/ab_libs.py $libs --rounds 3 > gpurun_out/ab_$TAG.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/ab_$TAG.log; exit 1; }
cat gpurun_out/ab_$TAG.log
for v in "$@"; do
  n=${v%%:*}; t=${v#$n}; t=${t#:}; o=pmc_${TAG}_$(echo $v | tr ':=,' '___')
  LDSO_AB_TUNE=$t LDSO_BA_LIB=$PWD/abl/$n/libldso_ba.so timeout -k 10 300 python tools/pmc_probe.py --kernel "k_linearize|k_point_sc" --out $o "FETCH_SIZE" "WRITE_SIZE" ${PMC_EXTRA:+"$PMC_EXTRA"} > gpurun_out/$o.log 2>&1 || { echo "pmc failed: $v"; tail -20 gpurun_out/$o.log; exit 1; }
  python -c "import json; d = json.load(open('gpurun_out/$o.json')); print('$v', {k: {c: round(x) for c, x in y.items()} for k, y in d.items()})"
done
echo done
