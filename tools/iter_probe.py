"""One S7 window: host-clock time of a GN iteration through ldso_ba_iterate (captured graph or
direct launches) against the host-solve path (linearize, ldso_ba_solve, resubstitute)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401

from ldso_amd import BAContext, synth

w = synth.make_window(**synth.S7, seed=1)
ns = w.nullspaces()
c = BAContext(0)
c.load([w])
reps = 200


def timeit(f):
    for _ in range(20):
        f()
    c.sync()
    t = time.perf_counter()
    for _ in range(reps):
        f()
    c.sync()
    return 1e3 * (time.perf_counter() - t) / reps


def host():
    c.linearize()
    x = c.solve(0, 2, 1e-5, ns)
    c.resubstitute(0, x, 1e-5, fetch=True)


out = {}
out["host_solve"] = timeit(host)
out["iterate_graph"] = timeit(lambda: c.iterate(2, 1e-5, [ns]))
out["iterate_graph_nosteps"] = timeit(lambda: c.iterate(2, 1e-5, [ns], fetch_steps=False))
os.environ["LDSO_BA_NO_GRAPH"] = "1"
out["iterate_direct"] = timeit(lambda: c.iterate(2, 1e-5, [ns]))
del os.environ["LDSO_BA_NO_GRAPH"]
os.environ["LDSO_BA_ITERATE_GRAPH"] = "1"
out["iterate_graph_env"] = timeit(lambda: c.iterate(2, 1e-5, [ns]))
del os.environ["LDSO_BA_ITERATE_GRAPH"]
out["pass_only"] = timeit(lambda: c.linearize())
out["optimize6"] = timeit(lambda: c.optimize(6, nullspaces=[ns]))
os.environ["LDSO_BA_NO_GRAPH"] = "1"
out["optimize6_direct"] = timeit(lambda: c.optimize(6, nullspaces=[ns]))
del os.environ["LDSO_BA_NO_GRAPH"]
print({k: round(v, 4) for k, v in out.items()})
