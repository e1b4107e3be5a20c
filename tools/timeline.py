"""Per-kernel durations and the gaps between consecutive kernels of the LAST optimize call in a
rocprofv3 kernel_trace.csv: python tools/timeline.py path/to/kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last optimize call = from the last k_keep_energy-led sequence start; take the last 80 kernels
tail = rows[-int(sys.argv[2]) if len(sys.argv) > 2 else -70:]
prev_end = None
tot_k = tot_g = 0
for r in tail:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3 if prev_end else 0.0
    import re
    m = re.search(r"(k_[a-z_]+)", r["Kernel_Name"])
    name = m.group(1) if m else r["Kernel_Name"][:40]
    print(f"{name:42s} {((e - s) / 1e3):8.2f} us   gap {gap:8.2f} us")
    tot_k += (e - s) / 1e3
    tot_g += gap
    prev_end = e
print(f"kernels {tot_k:.1f} us, gaps {tot_g:.1f} us")
