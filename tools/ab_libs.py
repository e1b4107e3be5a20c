"""A/B whole library builds on the bench workload: each build runs in its own process
(LDSO_BA_LIB=<path>), k_linearize / per-kernel HIP-event times, rounds interleaved.
  python tools/ab_libs.py lib1.so lib2.so[:key=value,...] ... [--windows 64] [--rounds 3]"""
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
B = WINDOWS
ws = [synth.make_window(**synth.S7, seed=1000 + i) for i in range(B)]
if IMAGE_ORDER:
    ws = [synth.in_image_order(w) for w in ws]
c = BAContext(0)
for kv in filter(None, os.environ.get("LDSO_AB_TUNE", "").split(",")):
    k, v = kv.split("=")
    c.set_tuning(int(k), int(v))
c.load(ws)
for _ in range(3):
    c.linearize()
out = {}
for acc in (True, False):
    c.linearize(accumulate=acc)
    c.set_kernel_timing(True)
    for _ in range(20):
        c.linearize(accumulate=acc)
    c.sync()
    kt = c.kernel_times()
    c.set_kernel_timing(False)
    out["acc" if acc else "noacc"] = {k: 1e3 * v[0] / v[1] for k, v in kt.items() if v[1]}
import time
for _ in range(5):
    c.linearize()
c.sync()
t0 = time.perf_counter()
for _ in range(50):
    c.linearize()
c.sync()
out["wall"] = {"pass": 1e6 * (time.perf_counter() - t0) / 50}
print("RESULT " + json.dumps(out))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--windows", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--image-order", action="store_true", help="points in image row order (LDSO's)")
    a = ap.parse_args()
    code = CHILD.replace("ROOT", repr(ROOT)).replace("WINDOWS", str(a.windows)).replace(
        "IMAGE_ORDER", str(a.image_order))
    res = {l: [] for l in a.libs}
    for _ in range(a.rounds):
        for l in a.libs:
            path, _, tune = l.partition(":")  # lib.so:key=value,key=value -> set_tuning before load
            env = dict(os.environ, LDSO_BA_LIB=os.path.abspath(path), LDSO_AB_TUNE=tune)
            p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
            line = [x for x in p.stdout.splitlines() if x.startswith("RESULT ")]
            if p.returncode != 0 or not line:
                print(l, "FAILED", p.returncode, p.stderr[-2000:])
                sys.exit(1)
            res[l].append(json.loads(line[0][7:]))
    for l, rs in res.items():
        best = {}
        for r in rs:
            for mode, kt in r.items():
                for k, v in kt.items():
                    best[(mode, k)] = min(best.get((mode, k), 1e9), v)
        print(l, " ".join(f"{m}:{k}={v:.1f}us" for (m, k), v in sorted(best.items())))
        print("   rounds acc:k_linearize", " ".join(f"{r['acc']['k_linearize']:.1f}" for r in rs),
              "noacc:k_linearize", " ".join(f"{r['noacc']['k_linearize']:.1f}" for r in rs))


if __name__ == "__main__":
    main()
