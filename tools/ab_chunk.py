"""A/B the k_linearize chunk size (residuals per wave) on the bench workload."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ldso_amd import BAContext, synth  # noqa: E402

ws = [synth.make_window(**synth.S7, seed=1000 + i) for i in range(64)]
res = {}
for rnd in range(2):
    for chunk in (16, 32, 64):
        c = BAContext(0)
        c.set_tuning(6, chunk)
        c.load(ws)
        for _ in range(3):
            c.linearize()
        c.set_kernel_timing(True)
        for _ in range(20):
            c.linearize()
        kt = c.kernel_times()
        c.close()
        res.setdefault(chunk, []).append({k: round(1e3 * v[0] / v[1], 1) for k, v in kt.items() if v[1]})
for k, v in res.items():
    print(k, v)
