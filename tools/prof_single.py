"""rocprofv3 target: one S7 window's device GN loop (ldso_ba_optimize) and ldso_ba_iterate, in
both solve modes, so the kernel trace shows every launch of a one-window iteration."""
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401  (HIP runtime first, as bench.py)

from ldso_amd import BAContext, synth

w = synth.make_window(**synth.S7, seed=1)
ns = [w.nullspaces()]
for exact in (0, 1):
    c = BAContext(0)
    c.set_tuning(12, exact)
    c.load([w])
    for _ in range(20):
        c.optimize(6, nullspaces=ns)
    for _ in range(20):
        c.iterate(2, 1e-5, ns)
    c.close()
print("done")
