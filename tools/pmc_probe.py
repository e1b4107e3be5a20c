"""Per-kernel PMC counters of the bench workload, one rocprofv3 --pmc pass per group.
  python tools/pmc_probe.py [--kernel REGEX] "SQ_WAVES SQ_WAVE_CYCLES ..." "FETCH_SIZE" ...
Prints the mean value per dispatch for every ldso kernel (first launch of each dropped).
Each pass runs under its own 120 s SIGKILL limit; an over-subscribed block hangs rocprofv3."""
import argparse
import collections
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ap = argparse.ArgumentParser()
ap.add_argument("--kernel", default="k_")
ap.add_argument("--windows", type=int, default=64)
ap.add_argument("--out", default="pmcprobe")
ap.add_argument("groups", nargs="+")
a = ap.parse_args()
out_root = os.path.join(ROOT, "gpurun_out", a.out)
allres = collections.defaultdict(dict)
for gi, grp in enumerate(a.groups):
    d = os.path.join(out_root, f"g{gi}")
    os.makedirs(d, exist_ok=True)
    cmd = ["timeout", "-s", "KILL", "120", "rocprofv3", "--pmc"] + grp.split() + [
        "--kernel-include-regex", a.kernel, "-d", d, "-o", "run", "--output-format", "csv", "--",
        sys.executable, os.path.join(ROOT, "tools", "pmc_driver.py"), "--steps", "4", "--windows", str(a.windows)]
    p = subprocess.run(cmd, env=dict(os.environ, TMPDIR="/tmp"), capture_output=True, text=True)
    if p.returncode != 0:
        print("group failed:", grp, p.returncode, p.stderr[-600:], flush=True)
        continue
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            name = row["Kernel_Name"]
            k = name.split("::")[-1].split("(")[0].split("<")[0] if "::" in name else name.split("(")[0]
            grid = int(row.get("Grid_Size", row.get("Grid_Size_X", "0")) or 0)
            vals[(f"{k}@{grid}", row["Counter_Name"])].append(float(row["Counter_Value"]))
    for (k, cn), v in vals.items():
        v = v[1:] if len(v) > 1 else v
        allres[k][cn] = sum(v) / len(v)
    print("group ok:", grp, flush=True)
print(json.dumps(allres, indent=1))
with open(os.path.join(ROOT, "gpurun_out", a.out + ".json"), "w") as f:
    json.dump(allres, f, indent=1)
