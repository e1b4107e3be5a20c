"""Per-kernel PMC counters of the bench workload, one rocprofv3 --pmc pass per group.
  python tools/pmc_probe.py "SQ_WAVES SQ_WAVE_CYCLES ..." "FETCH_SIZE" ...
Prints the mean value per dispatch for every ldso kernel (first launch of each dropped)."""
import collections
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out_root = os.path.join(ROOT, "gpurun_out", "pmcprobe")
allres = collections.defaultdict(dict)
for gi, grp in enumerate(sys.argv[1:]):
    d = os.path.join(out_root, f"g{gi}")
    os.makedirs(d, exist_ok=True)
    cmd = ["rocprofv3", "--pmc"] + grp.split() + ["-d", d, "-o", "run", "--output-format", "csv", "--", sys.executable,
                                                  os.path.join(ROOT, "tools", "pmc_driver.py"), "--steps", "4"]
    p = subprocess.run(cmd, env=dict(os.environ, TMPDIR="/tmp"), capture_output=True, text=True, timeout=600)
    if p.returncode != 0:
        print("group failed:", grp, p.stderr[-600:])
        continue
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            name = row["Kernel_Name"]
            if "::k_" not in name:
                continue
            k = name.split("::")[1].split("(")[0].split("<")[0]
            if int(row.get("Grid_Size", row.get("Grid_Size_X", "0")) or 0) < 20000 and k != "k_final":
                pass
            vals[(k, row["Counter_Name"])].append(float(row["Counter_Value"]))
    for (k, cn), v in vals.items():
        v = v[1:] if len(v) > 1 else v
        allres[k][cn] = sum(v) / len(v)
print(json.dumps(allres, indent=1))
with open(os.path.join(ROOT, "gpurun_out", "pmcprobe.json"), "w") as f:
    json.dump(allres, f, indent=1)
