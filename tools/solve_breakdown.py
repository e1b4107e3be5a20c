"""Time the parts of one single-window GN iteration (ms/solve): pass, system download, host
LDLT, resubstitute.  python tools/solve_breakdown.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ldso_amd import BAContext, synth  # noqa: E402

w = synth.make_window(**synth.S7, seed=1)
ns = w.nullspaces()
c = BAContext(0)
c.load([w])
for i in range(5):
    c.linearize()
    x = c.solve(0, i, 1e-5, ns)
    c.resubstitute(0, x, 1e-5)
reps = 50
T = {"linearize+sync": 0.0, "solve (download+LDLT)": 0.0, "resubstitute": 0.0, "system download": 0.0}
for _ in range(reps):
    t0 = time.perf_counter()
    c.linearize()
    c.sync()
    t1 = time.perf_counter()
    x = c.solve(0, 2, 1e-5, ns)
    t2 = time.perf_counter()
    c.resubstitute(0, x, 1e-5, fetch=True)
    t3 = time.perf_counter()
    T["linearize+sync"] += t1 - t0
    T["solve (download+LDLT)"] += t2 - t1
    T["resubstitute"] += t3 - t2
for _ in range(reps):
    c.linearize()
    c.sync()
    t0 = time.perf_counter()
    c.system(0)
    T["system download"] += time.perf_counter() - t0
print({k: round(1e3 * v / reps, 4) for k, v in T.items()}, "ms")
