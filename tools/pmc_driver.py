"""Workload driver for rocprofv3 counter passes: the bench's batched step, few iterations."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ldso_amd import BAContext, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--windows", type=int, default=64)
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--frames", type=int, default=7)
ap.add_argument("--points", type=int, default=2000)
a = ap.parse_args()
ws = [synth.make_window(n_frames=a.frames, n_points=a.points, seed=1000 + i) for i in range(a.windows)]
ctx = BAContext(0)
for kv in filter(None, os.environ.get("LDSO_AB_TUNE", "").split(",")):  # set_tuning before load (A/B)
    k, v = kv.split("=")
    ctx.set_tuning(int(k), int(v))
ctx.load(ws)
for w in ws:
    w.dI = None
for _ in range(a.steps):
    ctx.linearize()
ctx.sync()
n_gather = sum(int((ctx.residuals(i)["state"] != 1).sum()) for i in range(len(ws)))
print(f"n_gather={n_gather} residuals={ctx.stats()['residuals']}")
ctx.close()
