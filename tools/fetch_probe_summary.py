"""Summarise tools/gpu_fetch_probe.sh: per probe kernel the median counter values per launch against
the known bytes (every line of the 1-GiB buffer read once per launch, plus the 32-MiB line order)."""
import csv
import glob
import json
import os
import statistics
import sys

d = sys.argv[1]
nlines = 1024 * 1024 * 1024 // 128
perm_kib = nlines * 4 / 1024
vals = {}
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0].split("<")[-1].rstrip(">") or row["Kernel_Name"]
        vals.setdefault(k, {}).setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
out = {"lines_per_launch": nlines, "perm_kib_per_launch": perm_kib, "kernels": {}}
for k, cs in sorted(vals.items()):
    pieces = int(k) if k.isdigit() else None
    r = {c: statistics.median(v) for c, v in cs.items()}
    if pieces:
        req_kib = nlines * 16 * pieces / 1024 + perm_kib
        line_kib = nlines * 128 / 1024 + perm_kib
        r.update(requested_kib=req_kib, whole_line_kib=line_kib)
        if "FETCH_SIZE" in r:
            r["fetch_x1_over_whole_lines"] = r["FETCH_SIZE"] / line_kib
            r["fetch_x2_over_whole_lines"] = 2 * r["FETCH_SIZE"] / line_kib
            r["fetch_x1_over_requested"] = r["FETCH_SIZE"] / req_kib
    out["kernels"][f"pieces{pieces}" if pieces else k] = r
print(json.dumps(out, indent=1))
