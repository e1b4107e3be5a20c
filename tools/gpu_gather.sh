set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 tools/gather_probe 1024 > gpurun_out/gather.log 2>&1 || { cat gpurun_out/gather.log; exit 1; }
cat gpurun_out/gather.log
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/gather_pmc -o run --output-format csv -- tools/gather_probe 1024 > gpurun_out/gather_pmc.log 2>&1 || { tail gpurun_out/gather_pmc.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d gpurun_out/gather_pmc2 -o run --output-format csv -- tools/gather_probe 1024 > gpurun_out/gather_pmc2.log 2>&1 || { tail gpurun_out/gather_pmc2.log; exit 1; }
python3 - <<'PY'
import csv,glob,collections
for d in ("gather_pmc","gather_pmc2"):
    v=collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/{d}/**/*counter_collection.csv",recursive=True):
        for r in csv.DictReader(open(f)):
            v[(r["Kernel_Name"].split("(")[0],r["Counter_Name"])].append(float(r["Counter_Value"]))
    for k,x in sorted(v.items()): print(k, "mean %.0f"%(sum(x)/len(x)), "n", len(x))
PY
