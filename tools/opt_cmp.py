"""Bitwise comparison of ldso_ba_optimize between library builds: each build (LDSO_BA_LIB=<path>)
runs in its own process on the same windows (one S7 window; 6 S7 windows batched; an S11 window;
both solve modes) and every output of optimize() -- energies, frames, calibration, idepths,
iterations, statuses -- is compared bit for bit with the first build's.
  python tools/opt_cmp.py libA.so libB.so ..."""
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
cases = (("s7x1", [dict(synth.S7, seed=1000)]), ("s7x6", [dict(synth.S7, seed=1001 + i) for i in range(6)]),
         ("s11", [dict(n_frames=11, n_points=3000, seed=77)]))
for name, cfgs in cases:
    for exact in (0, 1):
        if exact and name == "s11":
            continue
        ws = [synth.make_window(**cf) for cf in cfgs]
        c = BAContext(0)
        c.set_tuning(12, exact)
        c.load(ws)
        for call in range(2):  # the second call replays the captured graph
            r = c.optimize(6, nullspaces=[w.nullspaces() for w in ws])
            for i, x in enumerate(r):
                xs = x if isinstance(x, list) else [x]
                for j, a in enumerate(xs):
                    a = np.ascontiguousarray(np.asarray(a))
                    out[f"{name}_e{exact}_c{call}_{i}_{j}"] = a.view(np.uint8).reshape(-1)
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
        diff = [k for k in res[0] if not np.array_equal(res[0][k], r[k])]
        print(f"{lib}: {len(res[0]) - len(diff)}/{len(res[0])} optimize outputs bit-identical to {libs[0]}", diff[:6])
        ok = ok and not diff
    print("ALL_IDENTICAL" if ok else "DIFFERENT")


if __name__ == "__main__":
    main()
