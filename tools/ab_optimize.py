"""A/B whole library builds on ldso_ba_optimize (one S7 window, and 64 of them): each build runs in
its own process (LDSO_BA_LIB=<path>), rounds interleaved, min over rounds of the mean host time
per optimize(6) call (all six iterations: th_opt_iterations = 0; the graph replayed).
  python tools/ab_optimize.py lib1.so[:key=value,...] lib2.so ... [--rounds 3] [--reps 20]"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, os, sys, time
sys.path.insert(0, ROOT)
import torch
torch.cuda.init()
from ldso_amd import BAContext, synth
from ldso_amd import _lib as L
out = {}
st = L.OptSettings.default(th_opt_iterations=0.0)
for B in (1, 64):
    ws = [synth.make_window(**synth.S7, seed=1000 + i) for i in range(B)]
    ns = [w.nullspaces() for w in ws]
    c = BAContext(0)
    for kv in filter(None, os.environ.get("LDSO_AB_TUNE", "").split(",")):
        c.set_tuning(*map(int, kv.split("=")))
    c.load(ws)
    for _ in range(3):  # the first call sets up and captures the graph
        c.optimize(6, nullspaces=ns, settings=st)
    c.sync()
    t0 = time.perf_counter()
    for _ in range(REPS):  # th = 0: six iterations whatever the state
        c.optimize(6, nullspaces=ns, settings=st)
    c.sync()
    out[f"optimize_{B}"] = 1e3 * (time.perf_counter() - t0) / REPS
    if B == 1:  # one linearize + accumulate pass
        for _ in range(5):
            c.linearize()
        c.sync()
        t0 = time.perf_counter()
        for _ in range(20 * REPS):
            c.linearize()
        c.sync()
        out["pass_1"] = 1e3 * (time.perf_counter() - t0) / (20 * REPS)
    c.close()
print("RESULT " + json.dumps(out))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    code = CHILD.replace("ROOT", repr(ROOT)).replace("REPS", str(a.reps))
    res = {l: [] for l in a.libs}
    for _ in range(a.rounds):
        for l in a.libs:
            path, _, tune = l.partition(":")
            env = dict(os.environ, LDSO_BA_LIB=os.path.abspath(path), LDSO_AB_TUNE=tune)
            p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
            line = [x for x in p.stdout.splitlines() if x.startswith("RESULT ")]
            if p.returncode != 0 or not line:
                print(l, "FAILED", p.returncode, p.stderr[-2000:])
                sys.exit(1)
            res[l].append(json.loads(line[0][7:]))
    for l, rs in res.items():
        print(l, " ".join(f"{k}={min(r[k] for r in rs):.3f}ms" for k in rs[0]))


if __name__ == "__main__":
    main()
