# One PMC group over several abl/<name> builds of the library (k_linearize by default).
# usage: tools/gpu_pmc_libs.sh TAG "COUNTERS" name1 name2 ...   (KRX=<regex> to pick the kernel)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1; CNT=$2; shift 2
for n in "$@"; do
  LDSO_BA_LIB=$PWD/abl/$n/libldso_ba.so timeout -k 10 200 python tools/pmc_probe.py --kernel "${KRX:-k_linearize}" --out pmc_${TAG}_$n "$CNT" > gpurun_out/pmc_${TAG}_$n.log 2>&1 || { echo "pmc failed: $n"; tail -20 gpurun_out/pmc_${TAG}_$n.log; exit 1; }
  python -c "import json; d = json.load(open('gpurun_out/pmc_${TAG}_$n.json')); print('$n', {k: {c: round(v) for c, v in x.items()} for k, x in d.items()})"
done
