"""Bitwise comparison of two library builds on the same pass: each build (LDSO_BA_LIB=<path>) runs
in its own process, linearises + accumulates a batch of synthetic windows and dumps the residual
outputs, the point terms and the assembled systems; the arrays are compared bit for bit.
  python tools/cmp_libs.py libA.so libB.so [--windows 8]"""
import argparse
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys
import numpy as np
sys.path.insert(0, ROOT)
from ldso_amd import BAContext, synth
ws = [synth.make_window(**synth.S7, seed=1000 + i) for i in range(WINDOWS)]
ws += [synth.make_window(n_frames=n, n_points=300, seed=77 + n) for n in (2, 5, 11, 16)]
c = BAContext(0)
c.load(ws)
c.linearize()
c.linearize()
out = {}
for w in range(len(ws)):
    for k, v in c.residuals(w).items():
        out[f"res{w}_{k}"] = np.asarray(v)
    for k, v in c.points(w).items():
        out[f"pt{w}_{k}"] = np.asarray(v)
    for k, v in c.system(w).items():
        out[f"sys{w}_{k}"] = np.asarray(v)
c.close()
np.savez(OUT, **out)
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs=2)
    ap.add_argument("--windows", type=int, default=8)
    a = ap.parse_args()
    dumps = []
    with tempfile.TemporaryDirectory() as td:
        for i, lib in enumerate(a.libs):
            out = os.path.join(td, f"d{i}.npz")
            code = CHILD.replace("ROOT", repr(ROOT)).replace("WINDOWS", str(a.windows)).replace("OUT", repr(out))
            env = dict(os.environ, LDSO_BA_LIB=os.path.abspath(lib))
            p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                print(lib, "FAILED", p.returncode, p.stderr[-3000:])
                sys.exit(1)
            dumps.append(dict(np.load(out)))
    d0, d1 = dumps
    bad = 0
    for k in sorted(d0):
        x, y = d0[k], d1[k]
        same = x.shape == y.shape and x.tobytes() == y.tobytes()
        if not same:
            bad += 1
            if bad <= 20:
                xf, yf = x.astype(np.float64).ravel(), y.astype(np.float64).ravel()
                rel = np.abs(xf - yf).max() / max(np.abs(xf).max(), 1e-300)
                print(f"DIFF {k}: {int((x != y).sum())} of {x.size} elements, max rel {rel:.2e}")
    print(f"{len(d0) - bad} of {len(d0)} arrays bitwise identical")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
