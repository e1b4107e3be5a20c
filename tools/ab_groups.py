"""A/B of the pipelined window groups (LDSO_BA_TUNE_PIPELINE_GROUPS) on the bench workload:
wall time per pass without kernel events."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ldso_amd import BAContext, synth  # noqa: E402

ws = [synth.make_window(**synth.S7, seed=1000 + i) for i in range(64)]
c = BAContext(0)
c.load(ws)
for rnd in range(2):
    for g in (1, 2, 4, 8):
        c.set_tuning(8, g)
        for _ in range(5):
            c.linearize()
        c.sync()
        t = time.perf_counter()
        for _ in range(50):
            c.linearize()
        c.sync()
        print(f"groups={g}: {1e3 * (time.perf_counter() - t) / 50:.4f} ms/pass")
