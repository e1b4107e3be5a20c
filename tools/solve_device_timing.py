"""Time ldso_ba_solve_device (all windows, x stays on device) at iteration 0 and 2."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ldso_amd import BAContext, synth  # noqa: E402
from ldso_amd import _lib as L  # noqa: E402

for B in (1, 64):
    ws = [synth.make_window(**synth.S7, seed=1000 + i) for i in range(B)]
    ns = [w.nullspaces() for w in ws]
    c = BAContext(0)
    c.load(ws)
    c.linearize()
    nsa = c._ns_all(ns)
    for it in (0, 2):
        for _ in range(3):
            L.check(c._lib.ldso_ba_solve_device(c._h, it, 1e-5, L.ptr(nsa, L.f64p), 7, L.ptr(None, L.f64p)))
        c.sync()
        t = time.perf_counter()
        for _ in range(20):
            L.check(c._lib.ldso_ba_solve_device(c._h, it, 1e-5, L.ptr(nsa, L.f64p), 7, L.ptr(None, L.f64p)))
        c.sync()
        print(f"windows={B} iteration={it}: {1e3 * (time.perf_counter() - t) / 20:.4f} ms per solve_device")
    c.close()
