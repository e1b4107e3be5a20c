"""A/B of whole library builds on the device solve alone: one S7 window (and 64), k_solve's
HIP-event time per launch, for iteration 0 and 2 (projection), each build in its own process.
  python tools/solve_ab.py lib1.so[:exact[:key=value,...]] lib2.so ... [--rounds 3]"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, os, sys
sys.path.insert(0, ROOT)
import torch
torch.cuda.init()
from ldso_amd import BAContext, synth
out = {}
for B in (1, 64):
    ws = [synth.make_window(**synth.S7, seed=1000 + i) for i in range(B)]
    ns = [w.nullspaces() for w in ws]
    c = BAContext(0)
    c.set_tuning(12, int(os.environ.get("LDSO_AB_EXACT", "0")))
    for kv in filter(None, os.environ.get("LDSO_AB_TUNE", "").split(",")):
        c.set_tuning(*map(int, kv.split("=")))
    c.load(ws)
    c.linearize()
    for it in (0, 2):
        for _ in range(5):
            c.solve_device(it, 1e-5, ns)
        c.set_kernel_timing(True)
        for _ in range(50):
            c.solve_device(it, 1e-5, ns)
        kt = c.kernel_times()
        c.set_kernel_timing(False)
        v = kt["k_solve"]
        out[f"w{B}_it{it}"] = 1e3 * v[0] / v[1]
    c.close()
print("RESULT " + json.dumps(out))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    code = CHILD.replace("ROOT", repr(ROOT))
    res = {l: [] for l in a.libs}
    for _ in range(a.rounds):
        for l in a.libs:
            path, _, rest = l.partition(":")
            exact, _, tune = rest.partition(":")
            env = dict(os.environ, LDSO_BA_LIB=os.path.abspath(path), LDSO_AB_EXACT=exact or "0", LDSO_AB_TUNE=tune)
            p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=200)
            line = [x for x in p.stdout.splitlines() if x.startswith("RESULT ")]
            if p.returncode != 0 or not line:
                print(l, "FAILED", p.returncode, p.stderr[-2000:])
                sys.exit(1)
            res[l].append(json.loads(line[0][7:]))
            print(l, line[0][7:], flush=True)
    for l, rs in res.items():
        print("BEST", l, " ".join(f"{k}={min(r[k] for r in rs):.1f}us" for k in rs[0]))


if __name__ == "__main__":
    main()
