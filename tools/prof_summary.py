"""Summarise a rocprofv3 kernel trace into a JSON of per-kernel launch counts and durations (us),
keyed by kernel name @ grid size (the batched and the one-window launches of a kernel apart):
  python tools/prof_summary.py SRC OUT.json [TITLE]
SRC is a directory holding run_kernel_trace.csv (--output-format csv) or a rocprofv3 SQLite
database (the `kernels` view)."""
import collections
import csv
import glob
import json
import os
import sqlite3
import sys


def rows_from(src):
    if os.path.isdir(src):
        for f in glob.glob(os.path.join(src, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
                yield r["Kernel_Name"], grid, int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    else:
        for name, s, e in sqlite3.connect(src).execute("select name, start, end from kernels order by start"):
            yield name, 0, s, e


def main():
    src, out = sys.argv[1], sys.argv[2]
    title = sys.argv[3] if len(sys.argv) > 3 else ""
    agg = collections.defaultdict(list)
    for name, grid, s, e in rows_from(src):
        n = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        agg[f"{n}@grid{grid}" if grid else n].append((e - s) / 1e3)
    res = {}
    for n, v in sorted(agg.items(), key=lambda x: -sum(x[1])):
        v2 = sorted(v)
        res[n] = {"launches": len(v), "total_us": round(sum(v), 2), "mean_us": round(sum(v) / len(v), 3),
                  "median_us": round(v2[len(v) // 2], 3), "min_us": round(v2[0], 3), "max_us": round(v2[-1], 3)}
    json.dump({"title": title, "source": "rocprofv3 --kernel-trace --stats", "kernels": res}, open(out, "w"), indent=1)
    for n, r in list(res.items())[:20]:
        print(f"{n[:48]:48s} n={r['launches']:5d} mean={r['mean_us']:8.2f} med={r['median_us']:8.2f} max={r['max_us']:8.2f}")


if __name__ == "__main__":
    main()
