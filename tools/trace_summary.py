"""Summarise a rocprofv3 --kernel-trace CSV per (kernel, grid size), so the batched bench
launches and the single-window launches of the same `bench.py` run are averaged separately.

  python tools/trace_summary.py gpurun_out/prof_TAG/run_kernel_trace.csv > profiles/rN_trace_summary.json
"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_[a-z_]+)", name)
    return m.group(1) if m else name.split("(")[0]


def main(path):
    groups = defaultdict(list)
    regs = {}
    for row in csv.DictReader(open(path)):
        k = (short(row["Kernel_Name"]), int(row["Grid_Size_X"]) * int(row["Grid_Size_Y"]) * int(row["Grid_Size_Z"]),
             int(row["Workgroup_Size_X"]))
        groups[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
        regs[k] = dict(vgpr=int(row["VGPR_Count"]), agpr=int(row["Accum_VGPR_Count"]), sgpr=int(row["SGPR_Count"]),
                       lds=int(row["LDS_Block_Size"]), scratch=int(row["Scratch_Size"]))
    out = []
    for (name, grid, wg), d in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        d.sort()
        out.append(dict(kernel=name, grid_threads=grid, workgroups=grid // wg, calls=len(d), avg_us=sum(d) / len(d),
                        median_us=d[len(d) // 2], min_us=d[0], max_us=d[-1], total_us=sum(d), **regs[(name, grid, wg)]))
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
