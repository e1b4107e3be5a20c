"""Summarise a rocprofv3 --kernel-trace CSV (run_kernel_trace.csv) into per-(kernel, grid) launch
counts and durations (us): python tools/prof_csv_summary.py TRACE.csv OUT.json [TITLE]"""
import collections
import csv
import json
import sys


def main():
    src, out = sys.argv[1], sys.argv[2]
    title = sys.argv[3] if len(sys.argv) > 3 else ""
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(src)):
        n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        agg[f"{n}@grid{r['Grid_Size_X']}"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    res = {}
    for n, v in sorted(agg.items(), key=lambda x: -sum(x[1])):
        v2 = sorted(v)
        res[n] = {"launches": len(v), "total_us": round(sum(v), 2), "mean_us": round(sum(v) / len(v), 3),
                  "median_us": round(v2[len(v2) // 2], 3), "min_us": round(v2[0], 3), "max_us": round(v2[-1], 3)}
    json.dump({"title": title, "source": "rocprofv3 --kernel-trace --stats", "kernels": res}, open(out, "w"), indent=1)
    for n, d in list(res.items())[:14]:
        print(f"{n[:64]:64s} {d['launches']:5d} mean={d['mean_us']:8.2f} med={d['median_us']:8.2f}")


if __name__ == "__main__":
    main()
