"""k_solve / GN-iteration timing of whole library builds (HIP events + host clock):
  python tools/solve_ab.py lib1.so lib2.so@LDSO_BA_SOLVE_LDS=1 ...   (each in its own process,
  LDSO_BA_LIB; '@NAME=VALUE' adds an environment variable to that process)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, sys, time
sys.path.insert(0, ROOT)
import torch
torch.cuda.init()
import numpy as np
from ldso_amd import BAContext, synth
from ldso_amd import _lib as L
out = {}
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
        c.set_kernel_timing(True)
        for _ in range(20):
            L.check(c._lib.ldso_ba_solve_device(c._h, it, 1e-5, L.ptr(nsa, L.f64p), 7, L.ptr(None, L.f64p)))
        kt = c.kernel_times()
        c.set_kernel_timing(False)
        out[f"B{B}_it{it}_k_solve_us"] = 1e3 * kt["k_solve"][0] / kt["k_solve"][1]
    if B == 1:
        for _ in range(5):
            c.iterate(0, 1e-5, ns)
        t = time.perf_counter()
        for _ in range(50):
            c.iterate(0, 1e-5, ns)
        out["B1_iterate_ms"] = 1e3 * (time.perf_counter() - t) / 50
    c.close()
print("RESULT " + json.dumps(out))
'''
for arg in sys.argv[1:]:
    lib, *extra = arg.split("@")
    env = dict(os.environ, LDSO_BA_LIB=os.path.abspath(lib))
    env.update(kv.split("=", 1) for kv in extra)
    p = subprocess.run([sys.executable, "-c", CHILD.replace("ROOT", repr(ROOT))], env=env, capture_output=True,
                       text=True, timeout=300)
    line = [x for x in p.stdout.splitlines() if x.startswith("RESULT ")]
    if p.returncode != 0 or not line:
        print(arg, "FAILED", p.stderr[-2000:])
        sys.exit(1)
    print(arg, {k: round(v, 4) for k, v in json.loads(line[0][7:]).items()})
