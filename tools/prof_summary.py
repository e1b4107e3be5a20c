"""Summarise a rocprofv3 kernel-trace database (prof_results.db: the `kernels` view) into a JSON
of per-kernel launch counts and durations (us): python tools/prof_summary.py DB OUT.json [TITLE]"""
import collections
import json
import sqlite3
import sys


def main():
    db, out = sys.argv[1], sys.argv[2]
    title = sys.argv[3] if len(sys.argv) > 3 else ""
    rows = sqlite3.connect(db).execute("select name, start, end from kernels order by start").fetchall()
    agg = collections.defaultdict(list)
    for name, s, e in rows:
        n = name.replace("void ", "").replace("(anonymous namespace)::", "")
        agg[n.split("(")[0]].append((e - s) / 1e3)
    res = {}
    for n, v in sorted(agg.items(), key=lambda x: -sum(x[1])):
        v2 = sorted(v)
        res[n] = {"launches": len(v), "total_us": round(sum(v), 2), "mean_us": round(sum(v) / len(v), 3),
                  "median_us": round(v2[len(v) // 2], 3), "min_us": round(v2[0], 3), "max_us": round(v2[-1], 3)}
    json.dump({"title": title, "source": "rocprofv3 --kernel-trace --stats", "kernels": res}, open(out, "w"), indent=1)
    for n, r in list(res.items())[:20]:
        print(f"{n[:40]:40s} n={r['launches']:5d} mean={r['mean_us']:8.2f} med={r['median_us']:8.2f} max={r['max_us']:8.2f}")


if __name__ == "__main__":
    main()
