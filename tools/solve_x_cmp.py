"""Bitwise comparison of the device solve's x between library builds: each build (LDSO_BA_LIB=<path>)
runs in its own process on the same windows (S7 and S11, iterations 0 and 2, the fast and the exact
mode) and the x vectors are compared bit for bit with the first build's.
  python tools/solve_x_cmp.py libA.so libB.so ..."""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys
sys.path.insert(0, ROOT)
import numpy as np
import torch
torch.cuda.init()
from ldso_amd import BAContext, synth
out = {}
for name, cfg, B in (("s7", synth.S7, 8), ("s11", dict(n_frames=11, n_points=3000), 3), ("n2", dict(n_frames=2, n_points=300), 2)):
    ws = [synth.make_window(**cfg, seed=500 + i) for i in range(B)]
    ns = [w.nullspaces() for w in ws]
    for exact in (0, 1):
        if exact and name == "s11":
            continue
        c = BAContext(0)
        c.set_tuning(12, exact)
        c.load(ws)
        c.linearize()
        for it in (0, 2):
            xs = c.solve_device(it, 1e-5, ns)
            for i, x in enumerate(xs):
                out[f"{name}_e{exact}_it{it}_w{i}"] = np.asarray(x)
        c.close()
np.savez(OUT, **out)
'''


def main():
    libs = sys.argv[1:]
    res = []
    with tempfile.TemporaryDirectory() as td:
        for k, lib in enumerate(libs):
            out = os.path.join(td, f"{k}.npz")
            env = dict(os.environ, LDSO_BA_LIB=os.path.abspath(lib))
            code = f"ROOT = {ROOT!r}\nOUT = {out!r}\n" + CHILD
            subprocess.run([sys.executable, "-c", code], env=env, check=True)
            res.append(dict(np.load(out)))
    ok = True
    for lib, r in zip(libs[1:], res[1:]):
        diff = [k for k in res[0] if not np.array_equal(res[0][k].view(np.uint64), r[k].view(np.uint64))]
        print(f"{lib}: {len(res[0]) - len(diff)}/{len(res[0])} x vectors bit-identical to {libs[0]}", diff[:6])
        ok = ok and not diff
    print("ALL_IDENTICAL" if ok else "DIFFERENT")


if __name__ == "__main__":
    main()
